#!/usr/bin/env python3
"""Writes tests/golden/films.npz and tests/golden/segments.npz from the CPU oracle, to freeze its
transport output: a later edit of the oracle (or of the kernel, which the GPU tests hold to the
oracle bit for bit) that changes any sample shows up against these files (tests/test_golden_films.py).

    python tools/make_golden_films.py

films.npz: 64x64 @ 4 spp films (float32 [64][64][4], XYZW) of
  cloud     c3 workload on the 64^3 procedural cloud (seed 10)
  constant  c2 workload on the constant 128^3 cube
  fire      c4 workload on the 64^3 cloud + 40*base temperature grid (seed 500)
segments.npz: RayMajorantIterator segments (log_majorant_trace rows, volume.cpp:176-192) of 8 rays
  through the 64^3 cloud ("cloud_<i>") and 4 through the sparse test grid ("sparse_<i>"), plus the
  rays themselves ("rays_cloud", "rays_sparse": origin xyz, direction xyz).
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

import oracle_lib as O  # noqa: E402
from grids import sparse_grid  # noqa: E402
from volume_path_tracer_amd.scenes import SynthGrid, workload  # noqa: E402

FILMS = {"cloud": ("c3", 64), "constant": ("c2", 128), "fire": ("c4", 64)}


def golden_film(name):
    wname, n = FILMS[name]
    wl = workload(wname, width=64, height=64, spp=4, grid_n=n)
    od = O.OracleGrid(SynthGrid(wl.density_kind, n).grid(), fix_majorants=True)
    ot = O.OracleGrid(SynthGrid(2, n).grid(), fix_majorants=False) if wl.temperature else None
    film, _, _ = O.render_jobs(wl.cfg, od, ot, 0, wl.cfg.jobs_per_wave() * 4)
    return film


def golden_rays():
    rng = np.random.default_rng(2024)
    o = np.array([[0.0, 0.0, -100.0]] * 8, np.float32)
    d = rng.normal(size=(8, 3)) * [0.2, 0.2, 0.0] + [0, 0, 1]
    cloud = np.concatenate([o, (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)], 1)
    o2 = np.array([[-40.0, -90.0, -700.0]] * 4, np.float32)
    d2 = rng.normal(size=(4, 3)) * [0.3, 0.3, 0.0] + [0, 0, 1]
    sparse = np.concatenate([o2, (d2 / np.linalg.norm(d2, axis=1, keepdims=True)).astype(np.float32)], 1)
    return cloud.astype(np.float32), sparse.astype(np.float32)


def golden_segments():
    cloud, sparse = golden_rays()
    out = {"rays_cloud": cloud, "rays_sparse": sparse}
    oc = O.OracleGrid(SynthGrid(1, 64).grid(), fix_majorants=True)
    os_ = O.OracleGrid(sparse_grid(), fix_majorants=True)
    for i, r in enumerate(cloud):
        out[f"cloud_{i}"] = O.majorant_trace(oc, r[:3], r[3:])
    for i, r in enumerate(sparse):
        out[f"sparse_{i}"] = O.majorant_trace(os_, r[:3], r[3:])
    return out


def main():
    g = ROOT / "tests" / "golden"
    np.savez_compressed(g / "films.npz", **{k: golden_film(k) for k in FILMS})
    np.savez_compressed(g / "segments.npz", **golden_segments())
    print("wrote", g / "films.npz", g / "segments.npz")


if __name__ == "__main__":
    main()
