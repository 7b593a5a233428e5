"""GPU parity of the PRODUCTION kernels (the ones bench.py times), not only the debug/records variant.

A launch whose jobs cover each pixel at most once adds exactly one fp32 atomic per film channel onto
zero, so the film IS the per-sample result: film[..., :3] == imaging_ratio * L and film[..., 3] == 1,
bit for bit.  Rendering single waves (or job ranges inside one wave) with the production kernels
therefore gives a bit-exact comparison with the oracle's per-sample records, for every kernel variant:

  <HasTemp=false, Runs=false>  C1 / C3 / C5 (the headline kernel)
  <HasTemp=false, Runs=true>   run skipping (chosen automatically for C2's constant cube; forced here
                               on the 128^3 cube and on a 64^3 cloud)
  <HasTemp=true,  Runs=false>  C4 (fire: blackbody emission from the temperature grid)
each as the throughput kernel and as the latency kernel (Lat: the lane's cold state in VGPRs; latency-bound
and partly filled launches -- C1, C2, small shares -- select it), forced with vpt_gpu_set_latency_kernel.

The production kernel's own event counters (samples, HDDA steps, density and temperature stencil
refreshes -- the terms of the algorithmic bytes) must equal the oracle's.
"""
import numpy as np
import pytest

import oracle_lib as O
from volume_path_tracer_amd import distributed as D
from volume_path_tracer_amd.scenes import SynthGrid, workload

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

COUNTERS = ("samples", "dda_steps", "stencils", "temp_stencils")


def _grids(wl):
    dens = SynthGrid(wl.density_kind, wl.grid_n).grid()
    temp = SynthGrid(2, wl.grid_n).grid() if wl.temperature else None
    return dens, temp


def _oracle_grids(dens, temp):
    od = O.OracleGrid(dens, fix_majorants=True)
    ot = O.OracleGrid(temp, fix_majorants=False) if temp is not None else None
    return od, ot


def records_film(cfg, jid_begin, count, rec):
    """The film of one sample per pixel, built from per-sample records (vpt_gpu_render_jobs_records
    layout): pixel (x0 + xl, y0 + yl) of job j holds imaging_ratio * rec[j * area + yl * rw + xl]."""
    W, H = cfg.width, cfg.height
    tw, th = int(cfg.tile_size[0]), int(cfg.tile_size[1])
    ntx = -(-W // tw)
    T = cfg.jobs_per_wave()
    area = tw * th
    film = np.zeros((H, W, 4), np.float32)
    r = np.float32(cfg.camera_parameters.imaging_ratio)
    for j in range(count):
        tile = (jid_begin + j) % T
        x0, y0 = (tile % ntx) * tw, (tile // ntx) * th
        rw, rh = min(W - x0, tw), min(H - y0, th)
        blk = rec[j * area: j * area + rw * rh].reshape(rh, rw, 3)
        if np.isnan(blk[:, :, 0]).all():
            continue  # single_pixel mode: no sample in this job
        film[y0:y0 + rh, x0:x0 + rw, :3] = r * blk
        film[y0:y0 + rh, x0:x0 + rw, 3] = 1.0
    return film


def _prod_film(it, jid_begin, count, stream=None):
    film = torch.zeros_like(it.film)
    it.render_jobs(jid_begin, count, film=film, stream=stream)
    torch.cuda.synchronize()
    return film.cpu().numpy()


def _assert_bitwise(a, b, what=""):
    diff = (a.view(np.uint32) != b.view(np.uint32)).any(axis=-1)
    assert not diff.any(), f"{what}: {int(diff.sum())} of {diff.size} pixels differ"


CASES = [
    # (workload, width, height, grid_n, run_skipping)
    ("c3", 48, 40, 64, 0),
    ("c3", 37, 29, 128, 0),
    ("c3", 48, 40, 64, 1),     # run skipping forced on a cloud (zero-majorant runs in its corners)
    ("c2", 64, 48, 128, 1),    # C2's constant cube: run skipping (its automatic choice)
    ("c2", 40, 32, 128, 0),    # ... and the plain kernel on it
    ("c4", 40, 32, 64, -1),    # temperature kernel
    ("c4", 56, 24, 128, -1),
]


@pytest.mark.parametrize("lat", [0, 1])
@pytest.mark.parametrize("name,w,h,n,runs", CASES)
def test_production_kernel_single_wave_films_bit_exact(name, w, h, n, runs, lat):
    """lat 0: the throughput kernels (7 / 6 waves per SIMD, cold state in LDS); lat 1: the latency kernels
    (cold state in VGPRs), which C1 / C2 select automatically."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload(name, width=w, height=h, spp=3, grid_n=n)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    it.set_latency_kernel(lat)
    if runs >= 0:
        it.set_run_skipping(runs)
    kv = it.kernel_variant()
    assert kv["has_temperature"] == wl.temperature and kv["run_skipping"] == (runs == 1)
    od, ot = _oracle_grids(dens, temp)
    T = wl.cfg.jobs_per_wave()
    it.counters(reset=True)
    tot = {k: 0 for k in COUNTERS}
    for wave in (1, 2, 3):
        f_g = _prod_film(it, (wave - 1) * T, T)  # a whole wave: cost-ordered scheduling
        f_o, _, c_o = O.render_jobs(wl.cfg, od, ot, (wave - 1) * T, T)
        _assert_bitwise(f_g, f_o, f"{name} wave {wave}")
        for k in COUNTERS:
            tot[k] += c_o[k]
    c = it.counters()
    for k in COUNTERS:
        assert c[k] == tot[k], (k, c[k], tot[k])


def test_run_skipping_is_the_automatic_choice_for_c2():
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c2", width=16, height=16, spp=1)
    it = Integrator(wl.cfg, *_grids(wl), device=0)
    assert it.kernel_variant()["run_skipping"]
    wl3 = workload("c3", width=16, height=16, spp=1, grid_n=128)
    assert not Integrator(wl3.cfg, *_grids(wl3), device=0).kernel_variant()["run_skipping"]


@pytest.mark.parametrize("runs", [0, 1])
def test_run_skipping_records_bit_exact(runs):
    """The debug twin of each density-only variant, per sample and per counter, on C2's cube."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c2", width=48, height=40, spp=2, grid_n=128)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    it.set_run_skipping(runs)
    jobs = wl.cfg.jobs_per_wave() * 2
    area = 64
    rec = torch.full((jobs * area, 3), float("nan"), device=it.dev)
    it.render_jobs(0, jobs, film=torch.zeros_like(it.film), records=rec)
    torch.cuda.synchronize()
    od, ot = _oracle_grids(dens, temp)
    _, r_o, c_o = O.render_jobs(wl.cfg, od, ot, 0, jobs, records=True)
    assert rec.cpu().numpy().tobytes() == r_o.tobytes()
    c = it.counters()
    for k in ("dda_steps", "segments", "draws", "stencils", "density_evals", "scatters", "shadow_rays",
              "rng_draws"):
        assert c[k] == c_o[k], k


def test_c1_full_workload_vs_oracle():
    """C1 at its real size (wdas_cloud 256x256, 4 spp, 512^3 stand-in): every sample of the 4 096 jobs
    bit-exact (records), each wave's production film bit-exact, the 4-wave film bit-exact (the ordered
    film: every pixel's samples added in wave order), and the counters equal."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c1")
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    od, ot = _oracle_grids(dens, temp)
    T = wl.cfg.jobs_per_wave()
    jobs = 4 * T
    f_o, r_o, c_o = O.render_jobs(wl.cfg, od, ot, 0, jobs, records=True)
    rec = torch.full((jobs * 64, 3), float("nan"), device=it.dev)
    it.render_jobs(0, jobs, film=torch.zeros_like(it.film), records=rec)
    torch.cuda.synchronize()
    assert rec.cpu().numpy().tobytes() == r_o.tobytes()
    for lat in (0, -1):  # the throughput kernel, and the latency kernel C1 selects
        it.set_latency_kernel(lat)
        it.counters(reset=True)
        for wave in range(4):
            f_g = _prod_film(it, wave * T, T)
            _assert_bitwise(f_g, records_film(wl.cfg, wave * T, T, r_o[wave * T * 64:(wave + 1) * T * 64]),
                            f"lat {lat} wave {wave + 1}")
        c = it.counters()
        for k in COUNTERS:
            assert c[k] == c_o[k], (lat, k)
        it.film.zero_()
        it.render_waves(1, 4)
        f_g = it.film_host()
        np.testing.assert_array_equal(f_g[..., 3], 4.0)
        _assert_bitwise(f_g, f_o, f"lat {lat} 4-wave film")


@pytest.mark.parametrize("lat", [0, 1])
@pytest.mark.parametrize("name", ["c3", "c4"])
def test_fullres_production_job_ranges_bit_exact(name, lat):
    """C3 / C4 at 1920x1080 on the 512^3 stand-ins: production-kernel films of job ranges spread over
    all 256 waves, bit-exact vs the oracle, and the stencil counters equal (throughput and latency kernels)."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload(name)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    it.set_latency_kernel(lat)
    od, ot = _oracle_grids(dens, temp)
    T = wl.cfg.jobs_per_wave()
    rng = np.random.default_rng(11 if name == "c3" else 12)
    begins = [int(w) * T + int(t) for w, t in zip(rng.integers(0, 256, 6), rng.integers(0, T - 200, 6))]
    it.counters(reset=True)
    tot = {k: 0 for k in COUNTERS}
    for b in begins:
        f_g = _prod_film(it, b, 160)
        f_o, _, c_o = O.render_jobs(wl.cfg, od, ot, b, 160)
        _assert_bitwise(f_g, f_o, f"jobs [{b}, {b + 160})")
        for k in COUNTERS:
            tot[k] += c_o[k]
    c = it.counters()
    for k in COUNTERS:
        assert c[k] == tot[k], (k, c[k], tot[k])
    if name == "c4":
        assert tot["temp_stencils"] > 0


def test_c5_4k_job_sample_bit_exact():
    """C5 (3840x2160, 1024 spp): jobs sampled across waves 1..1024 (jids up to 1.3e8), per-sample
    records and production films bit-exact vs the oracle."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c5")
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    od, ot = _oracle_grids(dens, temp)
    T = wl.cfg.jobs_per_wave()
    assert T == 480 * 270
    rng = np.random.default_rng(5)
    waves = sorted(set([0, 255, 256, 1023] + [int(x) for x in rng.integers(0, 1024, 4)]))
    for w in waves:
        b = w * T + int(rng.integers(0, T - 64))
        _, r_o, _ = O.render_jobs(wl.cfg, od, ot, b, 48, records=True)
        rec = torch.full((48 * 64, 3), float("nan"), device=it.dev)
        it.render_jobs(b, 48, film=torch.zeros_like(it.film), records=rec)
        f_g = _prod_film(it, b, 48)
        assert rec.cpu().numpy().tobytes() == r_o.tobytes(), f"wave {w + 1}"
        _assert_bitwise(f_g, records_film(wl.cfg, b, 48, r_o), f"wave {w + 1}")


def test_c5_strong_partitions_sum_to_one_launch_film():
    """The 8-GPU configuration's partition (distributed.rank_job_ranges, mode "strong"): for N = 2, 4, 8
    the ranks' job ranges cover the 1024 waves exactly once, and the per-rank films summed (the
    RCCL all-reduce) equal the one-launch film: sample counts exactly, XYZ/W to fp32 rounding
    (per-pixel RMSE far below north_star's 1e-4)."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c5")
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    T, spp = it.jobs_per_wave, wl.spp
    it.render_waves(1, spp)
    one = it.film_host().copy()
    np.testing.assert_array_equal(one[..., 3], spp)
    x1 = one[..., :3] / one[..., 3:]
    for N in (2, 4, 8):
        ranges = [D.rank_job_ranges(r, N, spp, T, "strong") for r in range(N)]
        flat = sorted(x for rr in ranges for x in rr)
        assert flat[0][0] == 0 and sum(n for _, n in flat) == spp * T
        assert all(a[0] + a[1] == b[0] for a, b in zip(flat, flat[1:]))
        total = torch.zeros_like(it.film)
        for rr in ranges:
            part = torch.zeros_like(it.film)
            for b, n in rr:
                it.render_jobs(b, n, film=part)
            total += part
        f = total.cpu().numpy()
        np.testing.assert_array_equal(f[..., 3], spp)
        xn = f[..., :3] / f[..., 3:]
        rmse = float(np.sqrt(np.mean((xn.astype(np.float64) - x1) ** 2)))
        assert rmse < 1e-5 and np.allclose(xn, x1, rtol=1e-4, atol=1e-6), (N, rmse)


def test_concurrent_launches_on_three_streams():
    """130 launches (more than the context's 64-slot counter ring) of small job ranges, round-robin on
    3 streams of one context, all in flight together into one film: every job renders exactly once
    (one wave: the film is bit-exact vs the oracle), and a set_tuning between launches waits for them."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c3", width=256, height=192, spp=1, grid_n=64)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    T = wl.cfg.jobs_per_wave()
    streams = [torch.cuda.Stream(device=it.dev) for _ in range(3)]
    film = torch.zeros_like(it.film)
    bounds = np.linspace(0, T, 131).astype(int)
    for i, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
        it.render_jobs(int(a), int(b - a), film=film, stream=streams[i % 3])
        if i == 64:
            it.set_tuning(gate_min=6)  # must not disturb the launches in flight
    torch.cuda.synchronize()
    od, ot = _oracle_grids(dens, temp)
    f_o, _, _ = O.render_jobs(wl.cfg, od, ot, 0, T)
    _assert_bitwise(film.cpu().numpy(), f_o, "3-stream film")


@pytest.mark.parametrize("lat", [0, 1])
@pytest.mark.parametrize("name", ["c3", "c4"])
def test_latency_launch_knobs_keep_films_bit_exact(name, lat):
    """Latency-bound launches (fewer jobs than grid lanes) spread their jobs over the wavefronts and run
    with their own gates (vpt_gpu_set_latency_tuning); a launch that fills the grid uses the normal
    path.  Every setting renders the oracle's single-wave films bit for bit, with equal counters."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload(name, width=48, height=40, spp=12, grid_n=64)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    it.set_latency_kernel(lat)
    od, ot = _oracle_grids(dens, temp)
    T = wl.cfg.jobs_per_wave()
    ref = [O.render_jobs(wl.cfg, od, ot, w * T, T) for w in range(2)]
    settings = [  # (wave_lanes, gate_min, gate_idle, gate_eval, gate_walk)
        (0, 1, 65, 1, 1),    # the defaults: auto spreading, every block runs for one lane
        (1, 1, 65, 1, 1),    # one lane per wavefront: some lanes take several jobs
        (5, 6, 8, 36, 4),    # the throughput gates
        (64, 2, 1, 64, 0),   # no spreading; evaluations only once no lane walks, one walk step per pass
    ]
    for s in settings:
        it.set_latency_tuning(*s)
        it.counters(reset=True)
        for w in range(2):
            _assert_bitwise(_prod_film(it, w * T, T), ref[w][0], f"{name} {s} wave {w + 1}")
        c = it.counters()
        for k in COUNTERS:
            assert c[k] == ref[0][2][k] + ref[1][2][k], (s, k)
    with pytest.raises(RuntimeError):
        it.set_latency_tuning(0, 1, 0, 1, 1)  # gate_idle 0 could stall a wavefront: rejected
    with pytest.raises(RuntimeError):
        it.set_tuning(gate_idle=0)
    # a grid of one block (256 lanes) that the 12 waves' 360 jobs fill: the throughput path
    it.set_tuning(grid_blocks=1)
    f_g = _prod_film(it, 0, 12 * T)
    f_o, _, _ = O.render_jobs(wl.cfg, od, ot, 0, 12 * T)
    np.testing.assert_array_equal(f_g[..., 3], 12.0)
    _assert_bitwise(f_g, f_o, "12 waves on one block")


@pytest.mark.parametrize("lat", [0, 1])
@pytest.mark.parametrize("case", ["small_voxels", "large_voxels", "unit_rotated"])
def test_mapped_grid_production_films_bit_exact(case, lat):
    """Non-identity maps (voxel size 0.05 / 20, anisotropic, rotated) through the production kernel:
    the walk-word prefetch's padding holds in index space whatever the voxel size, so the
    single-wave films equal the oracle's bit for bit and the counters agree."""
    from grids import MAPPED_CASES, mapped_grid, mapped_scene
    from volume_path_tracer_amd.render import Integrator

    _, scale, ang = next(c for c in MAPPED_CASES if c[0] == case)
    dens = mapped_grid(scale, ang)
    wl = workload("c3", width=64, height=48, spp=2, grid_n=64)
    mapped_scene(wl.cfg, 64 * max(scale), 1.0 / min(scale))
    it = Integrator(wl.cfg, dens, None, device=0)
    it.set_latency_kernel(lat)
    od = O.OracleGrid(dens, fix_majorants=True)
    T = wl.cfg.jobs_per_wave()
    it.counters(reset=True)
    tot = {k: 0 for k in COUNTERS}
    for wave in (1, 2):
        f_g = _prod_film(it, (wave - 1) * T, T)
        f_o, _, c_o = O.render_jobs(wl.cfg, od, None, (wave - 1) * T, T)
        _assert_bitwise(f_g, f_o, f"{case} wave {wave}")
        for k in COUNTERS:
            tot[k] += c_o[k]
    c = it.counters()
    for k in COUNTERS:
        assert c[k] == tot[k], (k, c[k], tot[k])


@pytest.mark.parametrize("lat", [0, 1])
def test_temperature_kernel_blackbody_from_memory_above_the_lds_rows(lat):
    """A temperature scale that reaches 20 000 K: the blackbody rows past the kernel's LDS copy
    (kBbLdsRows) are read from memory; the production films stay bit-exact vs the oracle."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c4", width=40, height=32, spp=2, grid_n=64)
    wl.cfg.volume_parameters.temperature_scale *= 10.0
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    it.set_latency_kernel(lat)
    od, ot = _oracle_grids(dens, temp)
    T = wl.cfg.jobs_per_wave()
    for wave in (1, 2):
        f_o, _, c_o = O.render_jobs(wl.cfg, od, ot, (wave - 1) * T, T)
        _assert_bitwise(_prod_film(it, (wave - 1) * T, T), f_o, f"wave {wave}")
    assert c_o["temp_stencils"] > 0



@pytest.mark.parametrize("lat", [0, 1])
@pytest.mark.parametrize("kind", ["shifted", "half_voxels", "sparse"])
def test_temperature_grid_of_another_map_or_topology(kind, lat):
    """The temperature kernel with a temperature grid whose map / topology differ from the density's
    (tests/grids.py temperature_pair): production films bit-exact vs the oracle, counters equal."""
    from grids import look_at, temperature_pair
    from volume_path_tracer_amd.render import Integrator

    dens, temp = temperature_pair(kind)
    wl = workload("c4", width=48, height=40, spp=2, grid_n=64)
    n = 128 if kind == "sparse" else 64
    look_at(wl.cfg, (0.3 * n, 0.6 * n, -2.2 * n), (0.5 * n, 0.45 * n, 0.5 * n))
    it = Integrator(wl.cfg, dens, temp, device=0)
    it.set_latency_kernel(lat)
    od, ot = _oracle_grids(dens, temp)
    T = wl.cfg.jobs_per_wave()
    it.counters(reset=True)
    tot = {k: 0 for k in COUNTERS}
    for wave in (1, 2):
        f_o, _, c_o = O.render_jobs(wl.cfg, od, ot, (wave - 1) * T, T)
        _assert_bitwise(_prod_film(it, (wave - 1) * T, T), f_o, f"{kind} wave {wave}")
        for k in COUNTERS:
            tot[k] += c_o[k]
    c = it.counters()
    for k in COUNTERS:
        assert c[k] == tot[k], (k, c[k], tot[k])
    assert tot["temp_stencils"] > 100


COMPACT_CASES = [
    # (workload, width, height, grid_n, run_skipping)
    ("c2", 96, 96, 128, 1),    # C2's cube with run skipping: the launch compaction targets
    ("c2", 80, 80, 128, 0),
    ("c3", 96, 80, 64, 0),     # the cloud
    ("c4", 96, 72, 64, -1),    # the temperature kernel (its temperature cell travels with the path)
]


@pytest.mark.parametrize("every", [1, 4, 16])
@pytest.mark.parametrize("name,w,h,n,runs", COMPACT_CASES)
def test_compacting_latency_kernel_films_bit_exact(name, w, h, n, runs, every):
    """Live-path compaction (vpt_gpu_set_compaction) on partly filled latency launches: a 4-block grid renders
    each wave's >= 64 jobs (more than 6 per wavefront: not a latency-bound launch), its four wavefronts meeting
    every 1 / 4 / 16 outer iterations to repack walking paths.  Each wave's film is the oracle's bit for bit,
    the event counters equal the oracle's, and the exchange ran (`exchanged` > 0)."""
    from volume_path_tracer_amd.render import Integrator

    wl = workload(name, width=w, height=h, spp=3, grid_n=n)
    dens, temp = _grids(wl)
    it = Integrator(wl.cfg, dens, temp, device=0)
    it.set_latency_kernel(1, 0)
    it.set_tuning(grid_blocks=4)
    it.set_compaction(every)
    if runs >= 0:
        it.set_run_skipping(runs)
    od, ot = _oracle_grids(dens, temp)
    T = wl.cfg.jobs_per_wave()
    assert T > 6 * 4 * 4  # partly filled, not latency-bound (kSpreadLanes x wavefronts)
    it.counters(reset=True)
    tot = {k: 0 for k in COUNTERS}
    for wave in (1, 2, 3):
        f_g = _prod_film(it, (wave - 1) * T, T)
        f_o, _, c_o = O.render_jobs(wl.cfg, od, ot, (wave - 1) * T, T)
        _assert_bitwise(f_g, f_o, f"{name} compact {every} wave {wave}")
        for k in COUNTERS:
            tot[k] += c_o[k]
    c = it.counters()
    for k in COUNTERS:
        assert c[k] == tot[k], (k, c[k], tot[k])
    assert c["exchanged"] > 0, c
