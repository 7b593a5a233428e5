"""GPU parity: the HIP integrator vs the CPU oracle at matched seeds (calls through the C ABI).

Bar: per-sample radiance bit-exact (records mode); films equal to within fp32 atomic-order
rounding (rtol 1e-5 on XYZ/W); the sample-count channel exact."""
import numpy as np
import pytest

import oracle_lib as O
from volume_path_tracer_amd.scenes import SynthGrid, workload

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _integrator(wl):
    from volume_path_tracer_amd.render import Integrator
    dens = SynthGrid(wl.density_kind, wl.grid_n).grid()
    temp = SynthGrid(2, wl.grid_n).grid() if wl.temperature else None
    return Integrator(wl.cfg, dens, temp, device=0), dens, temp


def _oracle(wl, dens, temp, jid_begin, count):
    od = O.OracleGrid(dens, fix_majorants=True)
    ot = O.OracleGrid(temp, fix_majorants=False) if temp is not None else None
    return O.render_jobs(wl.cfg, od, ot, jid_begin, count, records=True)


def _gpu_records(it, jid_begin, count):
    area = int(it.cfg.tile_size[0] * it.cfg.tile_size[1])
    rec = torch.full((count * area, 3), float("nan"), dtype=torch.float32, device=it.dev)
    film = torch.zeros_like(it.film)
    it.render_jobs(jid_begin, count, film=film, records=rec)
    torch.cuda.synchronize()
    return film.cpu().numpy(), rec.cpu().numpy()


@pytest.mark.parametrize("name,w,h,spp,n", [("c2", 40, 32, 2, 32), ("c3", 48, 40, 2, 64), ("c4", 40, 32, 2, 64),
                                             ("c1", 64, 48, 2, 128), ("c3", 37, 29, 3, 64)])
def test_gpu_records_bit_exact(name, w, h, spp, n):
    wl = workload(name, width=w, height=h, spp=spp, grid_n=n)
    it, dens, temp = _integrator(wl)
    jobs = wl.cfg.jobs_per_wave() * spp
    f_g, r_g = _gpu_records(it, 0, jobs)
    f_o, r_o, c_o = _oracle(wl, dens, temp, 0, jobs)
    same = (r_g.view(np.uint32) == r_o.view(np.uint32)).all(axis=1)
    assert same.all(), f"{(~same).sum()} of {same.size} samples differ"
    np.testing.assert_array_equal(f_g[..., 3], f_o[..., 3])
    np.testing.assert_allclose(f_g[..., :3], f_o[..., :3], rtol=1e-5, atol=1e-6)
    c = it.counters()
    assert c["samples"] == w * h * spp
    for k in ("dda_steps", "segments", "draws", "density_evals", "scatters", "shadow_rays", "rng_draws"):
        assert c[k] == c_o[k], k


def test_gpu_c3_fullres_job_sample_bit_exact():
    """C3 (1920x1080, 512^3 stand-in): jobs sampled across the whole jid space of 256 waves."""
    wl = workload("c3")
    it, dens, temp = _integrator(wl)
    T = it.jobs_per_wave
    rng = np.random.default_rng(0)
    begins = sorted(set(int(x) for x in rng.integers(0, 256 * T - 64, size=6))) + [T * 128 + T // 2]
    od = O.OracleGrid(dens, fix_majorants=True)
    diff = total = 0
    for b in begins:
        _, r_g = _gpu_records(it, b, 48)
        _, r_o, _ = O.render_jobs(wl.cfg, od, None, b, 48, records=True)
        ok = ~np.isnan(r_o[:, 0])
        diff += int((r_g[ok].view(np.uint32) != r_o[ok].view(np.uint32)).any(axis=1).sum())
        total += int(ok.sum())
    assert total > 0 and diff == 0, f"{diff}/{total}"


def test_gpu_c4_fullres_job_sample_bit_exact():
    """C4 (fire 1920x1080, 512^3 density + temperature): jobs sampled across the jid space, with the
    blackbody emission at every tentative collision."""
    wl = workload("c4")
    it, dens, temp = _integrator(wl)
    T = it.jobs_per_wave
    rng = np.random.default_rng(4)
    begins = sorted(set(int(x) for x in rng.integers(0, 256 * T - 64, size=5))) + [T * 200 + T // 2 + 7]
    od = O.OracleGrid(dens, fix_majorants=True)
    ot = O.OracleGrid(temp, fix_majorants=False)
    diff = total = emitting = 0
    for b in begins:
        _, r_g = _gpu_records(it, b, 48)
        _, r_o, _ = O.render_jobs(wl.cfg, od, ot, b, 48, records=True)
        ok = ~np.isnan(r_o[:, 0])
        diff += int((r_g[ok].view(np.uint32) != r_o[ok].view(np.uint32)).any(axis=1).sum())
        total += int(ok.sum())
        emitting += int((r_o[ok, 1] > 0).sum())
    assert total > 0 and emitting > 0 and diff == 0, f"{diff}/{total}"


def test_gpu_fire_lowscattering_scene_bit_exact():
    """The reference's third scene (scenes/fire_lowscattering.json) on the fire stand-in."""
    from volume_path_tracer_amd.scenes import Workload, _standin_camera, scene
    cfg = scene("fire_lowscattering")
    cfg.output_size[0], cfg.output_size[1], cfg.num_waves = 40, 24, 2
    _standin_camera(cfg, 800.0 * 64 / 512)
    wl = Workload("fire_lowscattering", cfg, 1, 64, True)
    it, dens, temp = _integrator(wl)
    jobs = cfg.jobs_per_wave() * 2
    f_g, r_g = _gpu_records(it, 0, jobs)
    f_o, r_o, _ = _oracle(wl, dens, temp, 0, jobs)
    same = (r_g.view(np.uint32) == r_o.view(np.uint32)).all(axis=1)
    assert same.all(), f"{(~same).sum()} of {same.size} samples differ"
    np.testing.assert_array_equal(f_g[..., 3], f_o[..., 3])


def test_gpu_sharded_waves_sum_to_full():
    """Wave-sharded rendering (the multi-GPU partition) reproduces the one-launch film."""
    wl = workload("c3", width=96, height=64, spp=8, grid_n=128)
    it, dens, temp = _integrator(wl)
    full = torch.zeros_like(it.film)
    it.render_waves(1, 8, film=full)
    parts = torch.zeros_like(it.film)
    for r in range(4):  # rank r of 4 renders waves r*2+1, r*2+2
        part = torch.zeros_like(it.film)
        it.render_waves(1 + 2 * r, 2, film=part)
        parts += part
    torch.cuda.synchronize()
    a, b = full.cpu().numpy(), parts.cpu().numpy()
    np.testing.assert_array_equal(a[..., 3], 8.0)
    np.testing.assert_allclose(a[..., :3], b[..., :3], rtol=1e-5, atol=1e-6)


def test_gpu_film_counts_and_determinism_c2_fullsize():
    """C2 at its BASELINE size (512x512, 64 spp): every pixel gets exactly 64 samples; two renders
    give the same film bit for bit (the ordered film); the analytic-side sanity: no NaN/Inf."""
    wl = workload("c2")
    it, dens, temp = _integrator(wl)
    it.render_waves(1, 64)
    f1 = it.film_host().copy()
    it.film.zero_()
    it.render_waves(1, 64)
    f2 = it.film_host()
    np.testing.assert_array_equal(f1[..., 3], 64.0)
    assert np.isfinite(f1).all()
    assert f1.tobytes() == f2.tobytes()


@pytest.mark.parametrize("gate_walk", [0, 1, 16, 64])
def test_gpu_sparse_grid_and_walk_loop_bit_exact(gate_walk):
    """Every HDDA level (gaps between lower nodes, upper/root/lower tiles) and every setting of the
    inner walk loop give the oracle's samples bit for bit."""
    from grids import look_at, sparse_grid

    from volume_path_tracer_amd.render import Integrator

    dens = sparse_grid()
    wl = workload("c3", width=64, height=48, spp=2)
    look_at(wl.cfg, (-40.0, -90.0, -700.0), (-40.0, -90.0, 10.0))
    wl.cfg.camera_parameters.vfov_deg = 50.0
    it = Integrator(wl.cfg, dens, None, device=0)
    it.set_tuning(gate_walk=gate_walk)
    jobs = wl.cfg.jobs_per_wave() * 2
    f_g, r_g = _gpu_records(it, 0, jobs)
    f_o, r_o, c_o = _oracle(wl, dens, None, 0, jobs)
    same = (r_g.view(np.uint32) == r_o.view(np.uint32)).all(axis=1)
    assert same.all(), f"{(~same).sum()} of {same.size} samples differ"
    c = it.counters()
    for k in ("dda_steps", "segments", "draws", "density_evals", "rng_draws"):
        assert c[k] == c_o[k], k


def test_gpu_film_rmse_within_north_star():
    """north_star: per-pixel RMSE < 1e-4 vs the reference at matched seeds.  Film XYZ/W over 16 spp
    (the fp32 atomic order differs from the serial oracle; every sample is bit-exact)."""
    wl = workload("c3", width=96, height=64, spp=16, grid_n=128)
    it, dens, temp = _integrator(wl)
    jobs = wl.cfg.jobs_per_wave() * 16
    it.render_jobs(0, jobs)
    f_g = it.film_host()
    od = O.OracleGrid(dens, fix_majorants=True)
    f_o, _, _ = O.render_jobs(wl.cfg, od, None, 0, jobs)
    np.testing.assert_array_equal(f_g[..., 3], f_o[..., 3])
    x_g, x_o = f_g[..., :3] / f_g[..., 3:], f_o[..., :3] / f_o[..., 3:]
    rmse = float(np.sqrt(np.mean((x_g.astype(np.float64) - x_o) ** 2)))
    assert rmse < 1e-4, rmse


def _records_equal(wl, dens, temp, jid_begin, count):
    from volume_path_tracer_amd.render import Integrator

    it = Integrator(wl.cfg, dens, temp, device=0)
    f_g, r_g = _gpu_records(it, jid_begin, count)
    f_o, r_o, c_o = _oracle(wl, dens, temp, jid_begin, count)
    assert r_g.tobytes() == r_o.tobytes()
    np.testing.assert_array_equal(f_g[..., 3], f_o[..., 3])
    return c_o


@pytest.mark.parametrize("case", ["tiles_only", "signed_values", "tiny_image", "odd_tiles", "no_jitter_single_pixel",
                                  "unaligned_jobs", "max_depth_0", "beyond_num_waves"])
def test_gpu_edge_cases_bit_exact(case):
    """Edge cases of the reference loop (worker.cpp:104-207) and of the tile/job mapping."""
    from grids import look_at, signed_grid, tiles_only_grid

    wl = workload("c3", width=24, height=16, spp=2, grid_n=64)
    dens = SynthGrid(1, 64).grid()
    begin, count = 0, None
    if case == "tiles_only":
        dens = tiles_only_grid()
        look_at(wl.cfg, (-500.0, 30.0, -300.0), (500.0, 30.0, 60.0))
    elif case == "signed_values":
        dens = signed_grid()
    elif case == "tiny_image":
        wl.cfg.output_size[0], wl.cfg.output_size[1] = 5, 3
    elif case == "odd_tiles":
        wl.cfg.output_size[0], wl.cfg.output_size[1] = 37, 23
        wl.cfg.tile_size[0], wl.cfg.tile_size[1] = 16, 3
    elif case == "no_jitter_single_pixel":
        wp = wl.cfg.worker_parameters
        wp.use_jitter = 0
        wp.single_pixel_enabled = 1
        wp.single_pixel_coord[0], wp.single_pixel_coord[1] = 11, 7
    elif case == "unaligned_jobs":
        begin, count = 7, 29
    elif case == "max_depth_0":
        wl.cfg.worker_parameters.max_depth = 0
    elif case == "beyond_num_waves":
        begin = wl.cfg.jobs_per_wave() * 5  # jobs past num_waves are valid jids (waves 6, 7)
    if count is None:
        count = wl.cfg.jobs_per_wave() * 2
    c = _records_equal(wl, dens, None, begin, count)
    if case == "max_depth_0":
        assert c["draws"] == 0 and c["scatters"] == 0
    if case == "tiles_only":
        assert c["draws"] > 0


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_gpu_job_order_modes_bit_exact(mode):
    """Every scheduling order renders the same samples (records keyed by jid) as the oracle."""
    from volume_path_tracer_amd import capi

    wl = workload("c3", width=48, height=40, spp=3, grid_n=64)
    it, dens, temp = _integrator(wl)
    it.set_job_order(mode)
    T = wl.cfg.jobs_per_wave()
    f_g, r_g = _gpu_records(it, T, 2 * T)  # waves 2..3: a whole-wave range not starting at 0
    f_o, r_o, c_o = _oracle(wl, dens, temp, T, 2 * T)
    assert r_g.tobytes() == r_o.tobytes()
    np.testing.assert_array_equal(f_g[..., 3], f_o[..., 3])
    np.testing.assert_allclose(f_g[..., :3], f_o[..., :3], rtol=1e-5, atol=1e-6)
    cost, rank = it.tile_costs()
    assert sorted(rank.tolist()) == list(range(T))
    assert np.all(np.diff(cost[rank]) <= 0) and cost.max() > 0 and capi.VPT_ORDER_COST_TAIL == 3
