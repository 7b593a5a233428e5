"""The device state machine (run on the CPU through tests/native/hostsim.cpp) reproduces the oracle
sample for sample, bit for bit: same RNG stream consumption, same float operations."""
import numpy as np
import pytest

import hostsim_lib as HS
import oracle_lib as O
from volume_path_tracer_amd.scenes import SynthGrid, workload


def _run_both(wl, jobs):
    dens = SynthGrid(wl.density_kind, wl.grid_n).grid()
    temp = SynthGrid(2, wl.grid_n).grid() if wl.temperature else None
    od = O.OracleGrid(dens, fix_majorants=True)
    ot = O.OracleGrid(temp, fix_majorants=False) if temp is not None else None
    f_o, r_o, c_o = O.render_jobs(wl.cfg, od, ot, 0, jobs, records=True)
    f_h, r_h, c_h = HS.render_jobs(wl.cfg, dens, temp, 0, jobs, records=True)
    return f_o, r_o, c_o, f_h, r_h, c_h


@pytest.mark.parametrize("name,w,h,spp,n", [("c2", 40, 32, 2, 32), ("c3", 48, 40, 2, 64), ("c4", 40, 32, 2, 64),
                                             ("c1", 24, 24, 3, 128)])
def test_records_bit_exact(name, w, h, spp, n):
    wl = workload(name, width=w, height=h, spp=spp, grid_n=n)
    jobs = wl.cfg.jobs_per_wave() * spp
    f_o, r_o, c_o, f_h, r_h, c_h = _run_both(wl, jobs)
    assert np.array_equal(r_o.view(np.uint32), r_h.view(np.uint32)), "per-sample radiance differs"
    assert np.array_equal(f_o.view(np.uint32), f_h.view(np.uint32))
    for k in ("samples", "dda_steps", "segments", "draws", "density_evals", "scatters", "shadow_rays", "rng_draws"):
        assert c_o[k] == c_h[k], k
    assert c_o["samples"] == w * h * spp


def test_single_pixel_and_no_jitter():
    wl = workload("c3", width=32, height=24, spp=2, grid_n=64)
    wp = wl.cfg.worker_parameters
    wp.single_pixel_enabled = 1
    wp.single_pixel_coord[0], wp.single_pixel_coord[1] = 17, 9
    wp.use_jitter = 0
    jobs = wl.cfg.jobs_per_wave() * 2
    f_o, r_o, c_o, f_h, r_h, c_h = _run_both(wl, jobs)
    assert c_o["samples"] == 2 and c_h["samples"] == 2
    assert np.array_equal(f_o.view(np.uint32), f_h.view(np.uint32))


def test_max_depth_and_zero_light():
    wl = workload("c3", width=24, height=16, spp=2, grid_n=64)
    wl.cfg.worker_parameters.max_depth = 3
    wl.cfg.worker_parameters.distant_light_multiplier = 0.0  # Li == 0: no NEE draws
    jobs = wl.cfg.jobs_per_wave() * 2
    f_o, r_o, c_o, f_h, r_h, c_h = _run_both(wl, jobs)
    assert c_o["shadow_rays"] == 0
    assert np.array_equal(r_o.view(np.uint32), r_h.view(np.uint32))


def test_sparse_grid_all_hdda_levels():
    """Rays crossing gaps between lower nodes, upper/root tiles and lower-node tiles: the HDDA
    dim changes (and the interior-cell fast path's boundaries) reproduce the oracle exactly."""
    from grids import look_at, sparse_grid

    dens = sparse_grid()
    wl = workload("c3", width=64, height=48, spp=2)
    look_at(wl.cfg, (-40.0, -90.0, -700.0), (-40.0, -90.0, 10.0))
    wl.cfg.camera_parameters.vfov_deg = 50.0
    od = O.OracleGrid(dens, fix_majorants=True)
    jobs = wl.cfg.jobs_per_wave() * 2
    f_o, r_o, c_o = O.render_jobs(wl.cfg, od, None, 0, jobs, records=True)
    f_h, r_h, c_h = HS.render_jobs(wl.cfg, dens, None, 0, jobs, records=True)
    assert np.array_equal(r_o.view(np.uint32), r_h.view(np.uint32))
    for k in ("dda_steps", "segments", "draws", "density_evals", "rng_draws"):
        assert c_o[k] == c_h[k], k
    # the scene is not trivially empty: many rays hit volume
    assert c_o["density_evals"] > 1000 and c_o["dda_steps"] > 5 * c_o["samples"]


def test_signed_values_grid():
    """Negative leaf values and negative / -0.0 tile values (majorants with the sign bit set) through
    the walk table's interior / edge / general paths."""
    from grids import signed_grid

    dens = signed_grid()
    wl = workload("c3", width=40, height=32, spp=2, grid_n=64)
    od = O.OracleGrid(dens, fix_majorants=True)
    jobs = wl.cfg.jobs_per_wave() * 2
    f_o, r_o, c_o = O.render_jobs(wl.cfg, od, None, 0, jobs, records=True)
    f_h, r_h, c_h = HS.render_jobs(wl.cfg, dens, None, 0, jobs, records=True)
    assert r_o.tobytes() == r_h.tobytes()
    for k in ("dda_steps", "segments", "draws", "density_evals", "rng_draws"):
        assert c_o[k] == c_h[k], k
    assert c_o["density_evals"] > 100


def test_tiles_only_grid():
    """A grid without leaves (upper/root/lower-node tiles only) through the device state machine."""
    from grids import look_at, tiles_only_grid

    dens = tiles_only_grid()
    wl = workload("c3", width=24, height=16, spp=2)
    look_at(wl.cfg, (-500.0, 30.0, -300.0), (500.0, 30.0, 60.0))
    od = O.OracleGrid(dens, fix_majorants=True)
    jobs = wl.cfg.jobs_per_wave() * 2
    f_o, r_o, c_o = O.render_jobs(wl.cfg, od, None, 0, jobs, records=True)
    f_h, r_h, c_h = HS.render_jobs(wl.cfg, dens, None, 0, jobs, records=True)
    assert r_o.tobytes() == r_h.tobytes()
    assert c_o["draws"] > 0 and c_o["draws"] == c_h["draws"]


@pytest.mark.parametrize("tail_waves", [0, 1, 3, -1])
@pytest.mark.parametrize("size", [(40, 24), (80, 72), (64, 64)])
def test_job_order_permutation_keeps_samples(tail_waves, size):
    """The kernel's cost-ordered scheduling (vpt_gpu_set_job_order) maps items onto the same jobs:
    with any tile ranking, every sample (keyed by its jid) is bit-identical to jid order.
    Tiles per wave: 15 (< one 64-tile group), 90 (one group + a ragged one), 64 (exactly one)."""
    wl = workload("c3", width=size[0], height=size[1], spp=3, grid_n=64)
    dens = SynthGrid(1, 64).grid()
    T = wl.cfg.jobs_per_wave()
    jobs = T * 3
    order = np.random.default_rng(5).permutation(T).astype(np.uint32)
    f_a, r_a, c_a = HS.render_jobs(wl.cfg, dens, None, T, jobs, records=True)
    f_b, r_b, c_b = HS.render_jobs(wl.cfg, dens, None, T, jobs, records=True, order=order, tail_waves=tail_waves)
    assert r_a.tobytes() == r_b.tobytes()
    np.testing.assert_array_equal(f_a[..., 3], f_b[..., 3])
    np.testing.assert_allclose(f_a[..., :3], f_b[..., :3], rtol=1e-5, atol=1e-6)
    assert c_a == c_b


@pytest.mark.parametrize("case", [c[0] for c in __import__("grids").MAPPED_CASES])
def test_mapped_grids_and_walk_padding(case):
    """Non-identity maps (voxel sizes 0.05 and 20, anisotropic, rotated): the device state machine
    equals the oracle bit for bit, and no walk-table lookup falls outside the padded table -- the
    lookahead of RayMajorantIterator::next (volume.cpp:63) is 1.0001 along the index-space ray, so the
    padding argument does not depend on the voxel size."""
    from grids import MAPPED_CASES, mapped_grid, mapped_scene

    _, scale, ang = next(c for c in MAPPED_CASES if c[0] == case)
    dens = mapped_grid(scale, ang)
    wl = workload("c3", width=40, height=32, spp=2, grid_n=64)
    mapped_scene(wl.cfg, 64 * max(scale), 1.0 / min(scale))
    od = O.OracleGrid(dens, fix_majorants=True)
    jobs = wl.cfg.jobs_per_wave() * 2
    HS.walk_outside(reset=True)
    f_o, r_o, c_o = O.render_jobs(wl.cfg, od, None, 0, jobs, records=True)
    f_h, r_h, c_h = HS.render_jobs(wl.cfg, dens, None, 0, jobs, records=True)
    assert r_o.tobytes() == r_h.tobytes()
    for k in ("dda_steps", "segments", "draws", "density_evals", "rng_draws"):
        assert c_o[k] == c_h[k], k
    assert c_o["density_evals"] > 500 and c_o["scatters"] > 50, c_o
    assert HS.walk_outside() == 0


@pytest.mark.parametrize("scale", [1.0, 10.0])
def test_blackbody_rows_in_lds_or_memory(scale):
    """The temperature kernel reads the blackbody table's first kBbLdsRows rows from LDS when the grid's
    temperatures stay below them (the fire stand-in: T <= 2 020 K), else the whole table from memory
    (scale 10: T up to 20 200 K).  The host simulator's LDS path sees NaN past those rows, so a wrong
    bound would show here."""
    wl = workload("c4", width=32, height=24, spp=2, grid_n=64)
    wl.cfg.volume_parameters.temperature_scale *= scale
    jobs = wl.cfg.jobs_per_wave() * 2
    f_o, r_o, c_o, f_h, r_h, c_h = _run_both(wl, jobs)
    assert np.array_equal(r_o.view(np.uint32), r_h.view(np.uint32))
    assert c_o["temp_stencils"] > 100


@pytest.mark.parametrize("kind", ["same", "shifted", "half_voxels", "sparse"])
def test_temperature_grid_of_another_map_or_topology(kind):
    """The temperature sampler on grids whose map and topology differ from the density's (a shifted
    grid, half-size voxels, every HDDA level's tiles): bit-exact, counters equal.  (These cases were
    written for the r03 joint-pool experiment, tools/experiments/r03_joint_temperature.patch, whose
    two lookup paths they exercise; they stay as coverage of the temperature grid's own lookups.)"""
    from grids import look_at, temperature_pair

    dens, temp = temperature_pair(kind)
    wl = workload("c4", width=32, height=24, spp=2, grid_n=64)
    n = 128 if kind == "sparse" else 64
    look_at(wl.cfg, (0.3 * n, 0.6 * n, -2.2 * n), (0.5 * n, 0.45 * n, 0.5 * n))
    jobs = wl.cfg.jobs_per_wave() * 2
    od, ot = O.OracleGrid(dens, fix_majorants=True), O.OracleGrid(temp, fix_majorants=False)
    f_o, r_o, c_o = O.render_jobs(wl.cfg, od, ot, 0, jobs, records=True)
    f_h, r_h, c_h = HS.render_jobs(wl.cfg, dens, temp, 0, jobs, records=True)
    assert np.array_equal(r_o.view(np.uint32), r_h.view(np.uint32)), "per-sample radiance differs"
    assert np.array_equal(f_o.view(np.uint32), f_h.view(np.uint32))
    for k in ("temp_stencils", "density_evals", "rng_draws"):
        assert c_o[k] == c_h[k], k
    assert c_o["temp_stencils"] > 100, c_o


@pytest.mark.parametrize("runs", [0, 1])
def test_zero_run_walk_words_bit_exact(runs):
    """Zero-run walk words (kZeroRunMax): a step in empty space hands the next cell's word over
    without loading it.  With the Runs variant off (the cloud's production kernel) the walk must
    synthesise words, and the samples stay the oracle's bit for bit, in both variants."""
    import ctypes as C
    L = HS.lib()
    L.vpths_walk_loads.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_int]
    L.vpths_set_runs.argtypes = [C.c_int]
    wl = workload("c3", width=48, height=40, spp=2, grid_n=256)
    jobs = wl.cfg.jobs_per_wave() * 2
    loads, synth = C.c_uint64(), C.c_uint64()
    L.vpths_walk_loads(C.byref(loads), C.byref(synth), 1)
    L.vpths_set_runs(runs)
    try:
        f_o, r_o, c_o, f_h, r_h, c_h = _run_both(wl, jobs)
    finally:
        L.vpths_set_runs(-1)
    L.vpths_walk_loads(C.byref(loads), C.byref(synth), 1)
    assert np.array_equal(r_o.view(np.uint32), r_h.view(np.uint32)), "per-sample radiance differs"
    assert c_o["dda_steps"] == c_h["dda_steps"] and c_o["segments"] == c_h["segments"]
    if runs == 0:
        assert synth.value > 0.01 * (loads.value + synth.value), (loads.value, synth.value)
