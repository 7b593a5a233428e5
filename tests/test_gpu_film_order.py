"""The ordered film (vpt_gpu_set_film_order): multi-wave films bit-identical to the oracle's.

The reference's film receives each pixel's samples in wave order -- a tile's next wave is handed out only once
its previous wave is released (src/tile_provider.cpp:40-60) and a job adds every pixel's sample as it traces it
(src/worker.cpp:203-204) -- so its film is deterministic.  The production launches store each sample's L into
a per-launch buffer and vpt_film_order_kernel adds them pixel by pixel in wave order: every multi-wave film here
is compared with the oracle's (tests/oracle_lib.py render_jobs / render_pool: the restated worker loop, jid
order) BIT FOR BIT, on every kernel variant, split launches, partial job ranges, single-pixel mode, launches on
three streams, and C3 / C4 frames at 1920x1080.  The atomic mode stays within fp32 rounding.
"""
import numpy as np
import pytest

import oracle_lib as O
from volume_path_tracer_amd import capi
from volume_path_tracer_amd.scenes import SynthGrid, workload

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _grids(wl):
    dens = SynthGrid(wl.density_kind, wl.grid_n).grid()
    temp = SynthGrid(2, wl.grid_n).grid() if wl.temperature else None
    return dens, temp


def _oracle(dens, temp):
    return O.OracleGrid(dens, fix_majorants=True), (O.OracleGrid(temp, fix_majorants=False) if temp is not None else None)


def _film(it, jid_begin, count, stream=None):
    film = torch.zeros_like(it.film)
    it.render_jobs(jid_begin, count, film=film, stream=stream)
    torch.cuda.synchronize()
    return film.cpu().numpy()


def _assert_bitwise(a, b, what=""):
    diff = (a.view(np.uint32) != b.view(np.uint32)).any(axis=-1)
    assert not diff.any(), f"{what}: {int(diff.sum())} of {diff.size} pixels differ"


CASES = [
    # (workload, width, height, grid_n, run_skipping, waves)
    ("c3", 48, 40, 64, 0, 6),
    ("c3", 37, 29, 128, 0, 5),   # ragged tiles on both edges
    ("c2", 64, 48, 128, 1, 5),   # C2's cube, run skipping
    ("c4", 40, 32, 64, -1, 5),   # temperature kernel
]


@pytest.mark.parametrize("lat", [0, 1])
@pytest.mark.parametrize("name,w,h,n,runs,waves", CASES)
def test_multi_wave_film_bit_identical(name, w, h, n, runs, waves, lat):
    """One launch of `waves` whole waves (cost-ordered: jobs run in no particular order) == the oracle's film."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload(name, width=w, height=h, spp=waves, grid_n=n)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    it.set_latency_kernel(lat)
    if runs >= 0:
        it.set_run_skipping(runs)
    T = wl.cfg.jobs_per_wave()
    f_g = _film(it, 0, waves * T)
    f_o, _, _ = O.render_jobs(wl.cfg, *_oracle(dens, temp), 0, waves * T)
    np.testing.assert_array_equal(f_g[..., 3], float(waves))
    _assert_bitwise(f_g, f_o, f"{name} lat {lat}")
    info = it.film_order_info()
    assert info["mode"] == capi.VPT_FILM_ORDERED and info["ordered_launches"] >= 1 and info["atomic_launches"] == 0
    assert info["buffer_bytes"] >= waves * T * 64 * 12


@pytest.mark.parametrize("name", ["c3", "c4"])
def test_job_orders_on_a_full_launch_bit_identical(name):
    """The same-tile job order (VPT_ORDER_COST_SAME_TILE, the default of full ordered-film launches: a wavefront's
    lanes take one tile's jobs of consecutive waves) and the cost tail, on a launch that fills its grid (one block
    set by set_tuning: neither the partly filled rule nor the latency kernel applies), render the oracle's film
    bit for bit -- and so the same film as each other."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload(name, width=96, height=64, spp=70, grid_n=64)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    it.set_tuning(grid_blocks=1)
    T = wl.cfg.jobs_per_wave()
    f_o, _, _ = O.render_jobs(wl.cfg, *_oracle(dens, temp), 0, 70 * T)
    for mode in (capi.VPT_ORDER_COST_SAME_TILE, capi.VPT_ORDER_COST_TAIL, capi.VPT_ORDER_JID):
        it.set_job_order(mode)
        _assert_bitwise(_film(it, 0, 70 * T), f_o, f"{name} order {mode}")
    assert it.film_order_info()["atomic_launches"] == 0


@pytest.mark.parametrize("cap_jobs", ["two_waves", "ragged"])
def test_split_launches_keep_the_order(cap_jobs):
    """A sample-buffer cap below the launch's size splits it into consecutive launches -- whole waves (cost order
    kept) or ragged job counts -- and the film stays the oracle's bit for bit."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c3", width=48, height=40, spp=7, grid_n=64)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    T = wl.cfg.jobs_per_wave()
    per_job = 64 * 12
    it.set_film_order(capi.VPT_FILM_ORDERED, (2 * T if cap_jobs == "two_waves" else 17) * per_job)
    f_g = _film(it, 0, 7 * T)
    f_o, _, _ = O.render_jobs(wl.cfg, *_oracle(dens, temp), 0, 7 * T)
    _assert_bitwise(f_g, f_o, cap_jobs)
    launches = it.film_order_info()["ordered_launches"]
    assert T == 30 and launches == (4 if cap_jobs == "two_waves" else -(-7 * T // 17)), launches


def test_partial_job_ranges_and_single_pixel():
    """Job ranges that start and end inside waves (several waves of some tiles, one of others), and the
    single_pixel mode (worker.cpp:113-116: one pixel gets samples, the rest of the film stays zero)."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c4", width=40, height=32, spp=4, grid_n=64)
    dens, temp = _grids(wl)
    od, ot = _oracle(dens, temp)
    it = Integrator(wl.cfg, dens, temp, device=0)
    T = wl.cfg.jobs_per_wave()
    for b, n in ((7, 2 * T + 5), (T - 3, 3), (3 * T + 1, T - 2)):
        _assert_bitwise(_film(it, b, n), O.render_jobs(wl.cfg, od, ot, b, n)[0], f"jobs [{b}, {b + n})")
    wl.cfg.worker_parameters.single_pixel_enabled = 1
    wl.cfg.worker_parameters.single_pixel_coord[0] = 13
    wl.cfg.worker_parameters.single_pixel_coord[1] = 21
    it1 = Integrator(wl.cfg, dens, temp, device=0)
    f_g = _film(it1, 0, 4 * T)
    f_o, _, _ = O.render_jobs(wl.cfg, od, ot, 0, 4 * T)
    _assert_bitwise(f_g, f_o, "single pixel")
    assert f_g[21, 13, 3] == 4.0 and f_g[..., 3].sum() == 4.0


def test_three_streams_run_in_enqueue_order():
    """Launches of consecutive slices of 3 waves enqueued round-robin on three streams of one context: ordered
    launches share the context's sample buffer, so each waits for the previous one's film pass -- they run in
    enqueue (jid) order and the film equals the oracle's 3-wave film bit for bit."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c3", width=256, height=192, spp=3, grid_n=64)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    T = wl.cfg.jobs_per_wave()
    streams = [torch.cuda.Stream(device=it.dev) for _ in range(3)]
    film = torch.zeros_like(it.film)
    bounds = np.linspace(0, 3 * T, 91).astype(int)
    for i, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
        it.render_jobs(int(a), int(b - a), film=film, stream=streams[i % 3])
    torch.cuda.synchronize()
    f_o, _, _ = O.render_jobs(wl.cfg, *_oracle(dens, temp), 0, 3 * T)
    _assert_bitwise(film.cpu().numpy(), f_o, "3-stream film")


def test_compacting_kernel_multi_wave_film():
    """Live-path compaction moves paths between threads (the job index travels in the cold state): the 3-wave
    film of a compacting launch is still the oracle's bit for bit."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c2", width=96, height=96, spp=3, grid_n=128)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    it.set_latency_kernel(1, 0)
    it.set_tuning(grid_blocks=4)
    it.set_compaction(4)
    T = wl.cfg.jobs_per_wave()
    it.counters(reset=True)
    f_g = _film(it, 0, 3 * T)
    assert it.counters()["exchanged"] > 0
    _assert_bitwise(f_g, O.render_jobs(wl.cfg, *_oracle(dens, temp), 0, 3 * T)[0], "compaction")


def test_atomic_mode_within_rounding_and_frees_the_buffer():
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c3", width=48, height=40, spp=6, grid_n=64)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    T = wl.cfg.jobs_per_wave()
    f_ord = _film(it, 0, 6 * T)
    assert it.film_order_info()["buffer_bytes"] > 0
    it.set_film_order(capi.VPT_FILM_ATOMIC)
    assert it.film_order_info()["buffer_bytes"] == 0
    f_at = _film(it, 0, 6 * T)
    info = it.film_order_info()
    assert info["atomic_launches"] == 1 and info["ordered_launches"] == 1
    np.testing.assert_array_equal(f_at[..., 3], f_ord[..., 3])
    np.testing.assert_allclose(f_at[..., :3], f_ord[..., :3], rtol=1e-5, atol=1e-6)
    with pytest.raises(RuntimeError):
        it.set_film_order(7)


@pytest.mark.parametrize("name", ["c3", "c4"])
def test_fullres_frame_waves_bit_identical_to_the_worker_pool(name):
    """C3 / C4 at 1920x1080 on the 512^3 stand-ins: waves 1..2 through the production path (one launch, cost
    order) against the oracle's worker pool (main.cpp:62-87 restated: threads over the restated TileProvider,
    whose wave gating orders each pixel's adds) -- bit for bit, counts included."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload(name)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    it.render_waves(1, 2)
    f_g = it.film_host()
    f_o, _, _ = O.render_pool(wl.cfg, *_oracle(dens, temp), 2, 16)
    _assert_bitwise(f_g, f_o, f"{name} waves 1..2")


def test_contexts_from_one_flatten():
    """vpt_gpu_create_many (the multi-GPU drop-in's setup): the grids flattened once and uploaded to each device --
    here two contexts on the box's one GPU.  Both render the oracle's 4-wave film bit for bit, and both report the
    same flatten time (one build)."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c4", width=40, height=32, spp=4, grid_n=64)
    dens, temp = _grids(wl)
    its = Integrator.create_many(wl.cfg, dens, temp, devices=(0, 0))
    T = wl.cfg.jobs_per_wave()
    f_o, _, _ = O.render_jobs(wl.cfg, *_oracle(dens, temp), 0, 4 * T)
    for it in its:
        _assert_bitwise(_film(it, 0, 4 * T), f_o, "create_many context")
    t0, t1 = (it.setup_timings() for it in its)
    assert t0["flatten_fix"] == t1["flatten_fix"] > 0 and t0["upload"] > 0
