"""Frozen transport output (tools/make_golden_films.py): 64x64 @ 4 spp films of the cloud, the
constant cube and the fire stand-ins, and RayMajorantIterator segment traces of 12 rays.

The oracle must reproduce them bit for bit (CPU), so an edit of the oracle that changes any sample is
caught even though the GPU tests hold the kernel to the oracle (they would drift together).  The GPU
kernel is checked against the same files directly: sample counts exactly, XYZ to fp32 atomic-order
rounding (4 adds per pixel), segment rows bit for bit."""
from pathlib import Path

import numpy as np
import pytest

from grids import sparse_grid
from volume_path_tracer_amd.scenes import SynthGrid

ROOT = Path(__file__).resolve().parents[1]
sys_path_tools = ROOT / "tools"
GOLD = ROOT / "tests" / "golden"


def _gen():
    import importlib.util

    spec = importlib.util.spec_from_file_location("make_golden_films", sys_path_tools / "make_golden_films.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("name", ["cloud", "constant", "fire"])
def test_oracle_reproduces_golden_film(name):
    want = np.load(GOLD / "films.npz")[name]
    got = _gen().golden_film(name)
    assert got.tobytes() == want.tobytes()


def test_oracle_reproduces_golden_segments():
    want = np.load(GOLD / "segments.npz")
    got = _gen().golden_segments()
    assert sorted(got) == sorted(want.files)
    for k in want.files:
        assert got[k].tobytes() == want[k].tobytes(), k


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cloud", "constant", "fire"])
def test_gpu_matches_golden_film(name):
    from volume_path_tracer_amd.render import Integrator
    from volume_path_tracer_amd.scenes import workload

    wname, n = _gen().FILMS[name]
    wl = workload(wname, width=64, height=64, spp=4, grid_n=n)
    temp = SynthGrid(2, n).grid() if wl.temperature else None
    it = Integrator(wl.cfg, SynthGrid(wl.density_kind, n).grid(), temp, device=0)
    it.render_waves(1, 4)
    got, want = it.film_host(), np.load(GOLD / "films.npz")[name]
    np.testing.assert_array_equal(got[..., 3], want[..., 3])
    np.testing.assert_allclose(got[..., :3], want[..., :3], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_gpu_matches_golden_segments():
    from volume_path_tracer_amd.render import Integrator
    from volume_path_tracer_amd.scenes import workload

    want = np.load(GOLD / "segments.npz")
    wl = workload("c3", width=8, height=8, spp=1, grid_n=64)
    for grid, key in ((SynthGrid(1, 64).grid(), "cloud"), (sparse_grid(), "sparse")):
        it = Integrator(wl.cfg, grid, None, device=0)
        for i, r in enumerate(want[f"rays_{key}"]):
            rows = it.majorant_trace(r[:3], r[3:])
            assert rows.tobytes() == want[f"{key}_{i}"].tobytes(), f"{key}_{i}"
