"""The reference-side drop-in (include/vpt_run.hpp) compiled and driven the way
main.cpp:62-87 drives vpt::run: several host threads, one shared TileProvider (restated with its wave
gating, tests/native/tile_provider_headless.hpp) and one shared host film, either
  * mode=drain: one GPU context per thread (vpt_gpu_create) and vpt_gpu::drain, the volume from an
    .nvdb file through the C++ reader (vpt_grid_read_nvdb) or the synthetic stand-in, or
  * mode=run: vpt_gpu::run(params, vol, camera, provider, film, rng) with the reference's own argument
    types (tests/native/reference_types_headless.hpp), the volume as NanoGrid<float> bytes and the seed
    private to the RNG -- the call main.cpp:63-68 makes, with only the function name changed.

Bar: no hang (the harness runs under a timeout), every pixel's sample count equals the number of
waves rendered, and the film equals the oracle's serial render of the same job ids -- bit for bit through run()
(its ordered frame, DrainOptions::ordered_frame), to fp32 atomic-order rounding where several drain() threads share
the provider (their feeds add atomically)."""
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_lib as O
from conftest import assert_hip_untouched
from volume_path_tracer_amd.scenes import SCENE_DIR, SynthGrid, workload

ROOT = Path(__file__).resolve().parents[1]
HARNESS = ROOT / "tests" / "native" / "build" / "run_gpu_harness"


def _assert_bitwise(a, b):
    diff = (a.view(np.uint32) != b.view(np.uint32)).any(axis=-1)
    assert not diff.any(), f"{int(diff.sum())} of {diff.size} pixels differ from the oracle's film"


def _harness(tmp_path, scene, w, h, waves, threads, batch, grid_n=64, temperature=0, stop_after=0, env=None, **extra):
    import os

    assert_hip_untouched()
    out = tmp_path / "film.f32"
    config = scene if Path(str(scene)).is_absolute() else SCENE_DIR / scene
    args = [str(HARNESS), f"config={config}", f"out={out}", f"w={w}", f"h={h}", f"waves={waves}",
            f"threads={threads}", f"batch={batch}", f"grid_n={grid_n}", f"temperature={temperature}",
            f"stop_after={stop_after}"] + [f"{k}={v}" for k, v in extra.items()]
    r = subprocess.run(args, capture_output=True, text=True, timeout=120, env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr + r.stdout
    return np.fromfile(out, np.float32).reshape(h, w, 4), r.stdout


def _oracle_film(name, w, h, waves, grid_n=64):
    wl = workload(name, width=w, height=h, spp=waves, grid_n=grid_n)
    dens = SynthGrid(1, grid_n).grid()
    temp = SynthGrid(2, grid_n).grid() if wl.temperature else None
    od = O.OracleGrid(dens, fix_majorants=True)
    ot = O.OracleGrid(temp, fix_majorants=False) if temp is not None else None
    f, _, _ = O.render_jobs(wl.cfg, od, ot, 0, wl.cfg.jobs_per_wave() * waves)
    return f


def test_harness_binary_built():
    assert HARNESS.exists(), "build with __graft_entry__.build() (tests/native/Makefile)"


@pytest.mark.gpu
@pytest.mark.spawns
@pytest.mark.parametrize("direct_below", [0, 1])
@pytest.mark.parametrize("threads,batch", [(2, 37), (2, 1000), (4, 7)])
def test_run_gpu_threads_share_one_tile_provider(tmp_path, threads, batch, direct_below):
    """Batches smaller and larger than a wave (T = 45 tiles), several threads racing on one provider:
    the batches cross wave boundaries and interleave, which deadlocked the round-1 sketch.  direct_below 0:
    the frame is small (225 jobs), so drain renders it as jid-range launches; 1: through a feed."""
    w, h, waves = 72, 40, 5
    film, log = _harness(tmp_path, "wdas_cloud.json", w, h, waves, threads, batch, direct_below=direct_below)
    np.testing.assert_array_equal(film[..., 3], waves)
    ref = _oracle_film("c3", w, h, waves)
    np.testing.assert_allclose(film[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)
    assert f"{waves} waves started" in log


@pytest.mark.gpu
@pytest.mark.spawns
def test_drain_with_helper_threads(tmp_path):
    """Two helper threads take tokens for the driving thread (vpt_gpu::help, what run()'s threads that find
    every GPU driven do): every job lands in the driver's feeds exactly once."""
    w, h, waves = 72, 40, 6
    film, log = _harness(tmp_path, "wdas_cloud.json", w, h, waves, 1, 5, helpers=2)
    np.testing.assert_array_equal(film[..., 3], waves)
    ref = _oracle_film("c3", w, h, waves)
    np.testing.assert_allclose(film[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.spawns
@pytest.mark.parametrize("direct_below", [0, 1])
def test_run_gpu_fire_scene_batches_over_two_waves(tmp_path, direct_below):
    """Temperature grid (fire.json) and batches of two waves (jid-range launches / a feed)."""
    w, h, waves = 48, 32, 4
    T = (w // 8) * (h // 8)
    film, _ = _harness(tmp_path, "fire.json", w, h, waves, 3, 2 * T, temperature=1, direct_below=direct_below)
    np.testing.assert_array_equal(film[..., 3], waves)
    ref = _oracle_film("c4", w, h, waves)
    np.testing.assert_allclose(film[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.spawns
@pytest.mark.parametrize("direct_below", [0, 1])
def test_run_gpu_stop_at_next_wave(tmp_path, direct_below):
    """stop_at_next_wave() during wave 2 (tile_provider.cpp:107-110): wave 2 completes, wave 3 never
    starts, so every pixel holds exactly 2 samples and the film is the oracle's 2-wave film."""
    w, h, waves = 64, 40, 6
    T = (w // 8) * (h // 8)
    film, log = _harness(tmp_path, "wdas_cloud.json", w, h, waves, 2, 11, stop_after=T + 5, direct_below=direct_below)
    np.testing.assert_array_equal(film[..., 3], 2)
    ref = _oracle_film("c3", w, h, 2)
    np.testing.assert_allclose(film[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)
    assert "2 waves started" in log


def test_integration_doc_shows_the_drop_in_verbatim():
    """INTEGRATION.md §2 is the compiled, tested drop-in, not a sketch."""
    doc = (ROOT / "INTEGRATION.md").read_text()
    src = (ROOT / "include" / "vpt_run.hpp").read_text()
    assert src.strip() in doc


@pytest.mark.parametrize("device", [-1, pytest.param(0, marks=[pytest.mark.gpu, pytest.mark.spawns])])
@pytest.mark.parametrize("seed", [0, 10, 500, 4294967295])
def test_drop_in_recovers_the_private_seed(tmp_path, seed, device):
    """The reference's RandomNumberGenerator keeps its seed private (random.hpp:86-115): the drop-in
    finds it from the job-0 stream -- device 0: one launch over all 2^32 candidates (vpt_gpu_find_seeds,
    what run() uses; <= 50 ms), -1: host threads."""
    if device >= 0:
        assert_hip_untouched()
    scene = json.loads((SCENE_DIR / "wdas_cloud.json").read_text())
    scene["seed"] = seed
    p = tmp_path / "s.json"
    p.write_text(json.dumps(scene))
    r = subprocess.run([str(HARNESS), f"config={p}", f"out={tmp_path / 'x'}", "mode=seed", f"device={device}"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and f"seed 0 {seed} " in r.stdout, r.stdout + r.stderr
    ms = float(r.stdout.split(f"seed 0 {seed} ")[1].split()[0])
    print(f"seed {seed} device {device}: {ms} ms")
    if device >= 0:
        assert ms <= 50.0, ms


@pytest.mark.gpu
@pytest.mark.spawns
@pytest.mark.parametrize("ordered", [0, 1])
@pytest.mark.parametrize("ctxs", [2, 3])
def test_one_taker_drives_several_contexts(tmp_path, ctxs, ordered):
    """drain_devices (run()'s multi-GPU path): ONE thread takes every token and feeds 2-3
    contexts -- here all on the box's one GPU, each launch held to 8 blocks so the feeds run side by side (a
    full-grid feed would hold every CU until it is closed).  ordered=0: each context's pipeline gets a lane's worth
    first, then the least-loaded one each batch, and the film is the oracle's to fp32 atomic-order rounding (feeds
    add atomically).  ordered=1 (what run() does): each context owns a band of tiles and orders its pixels' samples
    at the end -- the film equals the oracle's bit for bit.  Every pipeline closes its feed (VPT_DRAIN_TRACE)."""
    import os

    assert_hip_untouched()
    w, h, waves = 128, 96, 40
    out = tmp_path / "film.f32"
    args = [str(HARNESS), f"config={SCENE_DIR / 'wdas_cloud.json'}", f"out={out}", f"w={w}", f"h={h}",
            f"waves={waves}", f"threads={ctxs}", "batch=256", "grid_n=64", "multi=1", "devices=1", "grid_blocks=8",
            "flush_ms=20", f"ordered={ordered}"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=120, env=dict(os.environ, VPT_DRAIN_TRACE="1"))
    assert r.returncode == 0, r.stderr + r.stdout
    assert r.stderr.count(" closed ") == ctxs, r.stderr  # every context's feed ran and closed
    film = np.fromfile(out, np.float32).reshape(h, w, 4)
    np.testing.assert_array_equal(film[..., 3], waves)
    ref = _oracle_film("c3", w, h, waves)
    if ordered:
        assert r.stderr.count(" frame_done ") == ctxs, r.stderr
        _assert_bitwise(film, ref)
    else:
        np.testing.assert_allclose(film[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.spawns
def test_one_taker_small_ordered_frame_on_several_contexts(tmp_path):
    """A frame smaller than one launch's lanes through drain_devices with the ordered frame: jid-range launches on
    the first context (parts on several would add into the film one after another) -- the oracle's film bit for
    bit."""
    assert_hip_untouched()
    w, h, waves = 48, 32, 3
    out = tmp_path / "film.f32"
    args = [str(HARNESS), f"config={SCENE_DIR / 'wdas_cloud.json'}", f"out={out}", f"w={w}", f"h={h}",
            f"waves={waves}", "threads=3", "batch=16", "grid_n=64", "multi=1", "devices=1", "grid_blocks=8", "ordered=1"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    film = np.fromfile(out, np.float32).reshape(h, w, 4)
    _assert_bitwise(film, _oracle_film("c3", w, h, waves))


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [1, 2, 8])
def test_mock_taker_rate_on_the_box(devices):
    """On the GPU box's own cores (no GPU used): one taker feeding 1 / 2 / 8 mock GPUs keeps >= 0.9x the rate
    of the provider alone on one thread (tests/test_dropin_protocol.py mock_rates)."""
    from test_dropin_protocol import mock_rates

    fr, pr = mock_rates(devices, runs=5)
    print(f"devices {devices}: frame {fr:.2f} provider {pr:.2f} M tokens/s ({fr / pr:.3f}x)")
    assert fr >= 0.9 * pr, (devices, fr, pr)


@pytest.mark.parametrize("w,h,tile,batch", [(72, 40, 8, 3), (70, 38, 8, 1), (70, 38, 16, 100), (4, 4, 8, 1),
                                            (20, 12, 8, 2), (64, 48, 8, 500)])
def test_drop_in_reads_the_tile_size_off_the_tokens(tmp_path, w, h, tile, batch):
    """TileProvider keeps its tile size private: the drop-in takes the largest rect of its first batch
    and checks every rect against the jid mapping (an image narrower than a tile gives the image width,
    which maps every jid the same way)."""
    scene = json.loads((SCENE_DIR / "wdas_cloud.json").read_text())
    scene["tile_size"] = [tile, tile]
    p = tmp_path / "t.json"
    p.write_text(json.dumps(scene))
    r = subprocess.run([str(HARNESS), f"config={p}", f"out={tmp_path / 'x'}", "mode=tiles", f"w={w}", f"h={h}",
                        "waves=2", f"batch={batch}"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    ok, tw, th, _ = (int(x) for x in r.stdout.split("tiles")[1].split())
    assert ok == 1 and tw == min(tile, w) and (th == min(tile, h) or batch < -(-w // tile)), r.stdout


def _write_buffer(tmp_path, grid, name):
    from volume_path_tracer_amd import nvdb

    p = tmp_path / f"{name}.grid"
    p.write_bytes(nvdb.buffer_from_grid(grid, name))
    return p


@pytest.mark.gpu
@pytest.mark.spawns
@pytest.mark.parametrize("feed", ["0", "1"])
@pytest.mark.parametrize("scene,name", [("wdas_cloud.json", "c3"), ("fire.json", "c4")])
def test_reference_signature_run_from_main_threads(tmp_path, scene, name, feed):
    """vpt_gpu::run with main.cpp's arguments from 3 worker threads on one GPU: one thread drives the
    device, the others return; the seed is recovered from the RNG (private in the reference); the
    tile size from the tokens; the grids are read from NanoGrid<float> memory.  The frame is small: jid-range
    launches (feed 0), or through a feed and its ordered frame (feed 1: VPT_DROPIN_DIRECT_BELOW=1)."""
    w, h, waves = 72, 40, 3
    extra = dict(mode="run", gridbuf=_write_buffer(tmp_path, SynthGrid(1, 64).grid(copy=True), "density"))
    if name == "c4":
        extra["tempbuf"] = _write_buffer(tmp_path, SynthGrid(2, 64).grid(copy=True), "temperature")
    film, log = _harness(tmp_path, scene, w, h, waves, 3, 0, env={"VPT_DROPIN_DIRECT_BELOW": feed}, **extra)
    np.testing.assert_array_equal(film[..., 3], waves)
    ref = _oracle_film(name, w, h, waves)
    _assert_bitwise(film, ref)  # (run()'s ordered frame: the reference's film bit for bit)
    assert f"{waves} waves started" in log


@pytest.mark.gpu
@pytest.mark.spawns
def test_reference_signature_run_three_frames_in_one_process(tmp_path):
    """Three run() calls in one process, each with a fresh provider and film (a caller rendering again): the host
    grid copies of one call are kept until the next (vpt_run.hpp) and every frame is the oracle's."""
    w, h, waves = 48, 32, 3
    extra = dict(mode="run", frames=3, gridbuf=_write_buffer(tmp_path, SynthGrid(1, 64).grid(copy=True), "density"),
                 tempbuf=_write_buffer(tmp_path, SynthGrid(2, 64).grid(copy=True), "temperature"))
    film, log = _harness(tmp_path, "fire.json", w, h, waves, 2, 0, env={"VPT_DROPIN_DIRECT_BELOW": "1"}, **extra)
    assert "frame 1 total_ms" in log and "frame 2 total_ms" in log
    np.testing.assert_array_equal(film[..., 3], waves)
    ref = _oracle_film("c4", w, h, waves)
    _assert_bitwise(film, ref)


@pytest.mark.gpu
@pytest.mark.spawns
@pytest.mark.parametrize("ordered", ["1", "0"])
def test_reference_signature_run_stop_at_next_wave(tmp_path, ordered):
    """run() with stop_at_next_wave() during wave 2 (tile_provider.cpp:107-110) through a feed (VPT_DROPIN_DIRECT_BELOW):
    every pixel holds exactly 2 samples and the film is the oracle's 2-wave film -- bit for bit with run()'s ordered
    frame (the frame ends before its waves do), to atomic-order rounding with VPT_DROPIN_ORDERED=0."""
    w, h, waves = 256, 160, 40
    T = (w // 8) * (h // 8)
    extra = dict(mode="run", gridbuf=_write_buffer(tmp_path, SynthGrid(1, 64).grid(copy=True), "density"))
    film, log = _harness(tmp_path, "wdas_cloud.json", w, h, waves, 2, 0, stop_after=T + 5,
                         env={"VPT_DROPIN_ORDERED": ordered, "VPT_DROPIN_DIRECT_BELOW": "1"}, **extra)
    np.testing.assert_array_equal(film[..., 3], 2)
    ref = _oracle_film("c3", w, h, 2)
    if ordered == "1":
        _assert_bitwise(film, ref)
    else:
        np.testing.assert_allclose(film[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.spawns
def test_drain_from_nvdb_file_with_tiles_at_every_level(tmp_path):
    """An .nvdb file (ZIP codec) of a grid with lower / upper / root tiles and sparse lower nodes, read
    by the C++ reader inside the harness and rendered by 2 threads, against the oracle on the grid."""
    from grids import sparse_grid
    from volume_path_tracer_amd import nvdb

    g = sparse_grid()
    path = tmp_path / "sparse.nvdb"
    nvdb.write_nvdb(path, {"density": g}, codec=nvdb.CODEC_ZIP)
    scene = json.loads((SCENE_DIR / "wdas_cloud.json").read_text())
    scene["camera_parameters"].update(position=[-40.0, -90.0, -700.0], look=[-40.0, -90.0, 10.0], up=[0.0, 1.0, 0.0],
                                      vfov_deg=50.0)
    cfg_path = tmp_path / "scene.json"
    cfg_path.write_text(json.dumps(scene))
    w, h, waves = 64, 48, 2
    film, _ = _harness(tmp_path, cfg_path, w, h, waves, 2, 50, nvdb=path, dist=0)
    np.testing.assert_array_equal(film[..., 3], waves)
    wl = workload("c3", width=w, height=h, spp=waves)
    from grids import look_at
    look_at(wl.cfg, (-40.0, -90.0, -700.0), (-40.0, -90.0, 10.0))
    wl.cfg.camera_parameters.vfov_deg = 50.0
    f_o, _, c = O.render_jobs(wl.cfg, O.OracleGrid(g, fix_majorants=True), None, 0, wl.cfg.jobs_per_wave() * waves)
    assert c["density_evals"] > 1000
    np.testing.assert_allclose(film[..., :3], f_o[..., :3], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.spawns
def test_library_before_torch_keeps_one_hip_runtime():
    """A process that reaches the C ABI (capi.lib()) before it imports torch still ends up with a single HIP
    runtime -- torch's -- and torch sees the GPU (r03zl: /opt/rocm's runtime loaded first made torch's second
    ROCr find no GPU on some boxes).  Run in a child process, the way a user script starts."""
    import subprocess
    import sys

    code = ("import sys; sys.path.insert(0, '.')\n"
            "from volume_path_tracer_amd.scenes import SynthGrid, workload\n"
            "wl = workload('c3', width=16, height=16, spp=1, grid_n=32)\n"
            "dens = SynthGrid(wl.density_kind, wl.grid_n).grid()\n"
            "import torch\n"
            "from volume_path_tracer_amd.render import Integrator\n"
            "it = Integrator(wl.cfg, dens, None, device=0)\n"
            "it.render_jobs(0, wl.cfg.jobs_per_wave())\n"
            "torch.cuda.synchronize()\n"
            "libs = {l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}\n"
            "print('runtimes', len(libs), 'samples', it.counters()['samples'])\n")
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "runtimes 1 samples 256" in r.stdout, r.stdout


@pytest.mark.gpu
@pytest.mark.spawns
def test_progressive_film_rises_during_the_drain(tmp_path):
    """What main.cpp's 5-FPS window shows (main.cpp:101-132): while the drain renders a full C3 frame
    (1920x1080, 256 waves, 512^3 stand-in), a thread samples the host film every 10 ms.  With a film snapshot
    every 50 ms the film's sample count rises monotonically through several intermediate values, never ahead
    of the jobs handed out, and ends with every pixel at 256 samples.  (flush_ms: the film thread's snapshot
    period.)"""
    w, h, waves = 1920, 1080, 256
    film, log = _harness(tmp_path, "wdas_cloud.json", w, h, waves, 1, 4096, grid_n=512, flush_ms=50, sample_ms=10)
    samples = [tuple(float(v) for v in line.split()[1:4]) for line in log.splitlines() if line.startswith("sample ")]
    assert len(samples) >= 10, log[-2000:]
    in_film = [s[2] for s in samples]
    assert all(b >= a for a, b in zip(in_film, in_film[1:])), in_film
    assert all(s[2] <= s[1] + 1e-6 for s in samples), samples  # the film never shows jobs not yet handed out
    assert len({v for v in in_film if 0.0 < v < waves}) >= 3, in_film
    assert (film[..., 3] == waves).all()


@pytest.mark.gpu
@pytest.mark.spawns
def test_drain_with_a_small_backlog_never_stalls(tmp_path):
    """Full C4 frames with the pusher's backlog at a quarter of the lanes (98 304): the launch's first lane's
    worth of reservations lands its backlog hints in any order, and before r05 the one hint word could keep an
    early value for good -- a backlog that read full while every lane waited, one run in ~5 hanging (r05q).
    Now 6 frames in a row complete and count every sample."""
    w, h, waves = 1920, 1080, 256
    film, log = _harness(tmp_path, "fire.json", w, h, waves, 1, 4096, grid_n=512, temperature=1, backlog=98304,
                         frames=6)
    assert log.count("render_ms") == 6, log[-2000:]
    assert (film[..., 3] == waves).all()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["full_grid", "small_grid", "staged_small_grid"])
def test_feed_renders_pushed_jobs_in_any_order(mode):
    """vpt_gpu_feed_*: job ids pushed out of order and with gaps render the oracle's samples; the close (or,
    for a staged feed, the collect) adds exactly the pushed jobs' sample counts.  Two feeds of one context on
    two streams, the second opened while the first runs (its lanes start as the first's leave, once it is
    closed).  full_grid: the ~2 000 jobs are fewer than the launch's lanes, so it starts at close.
    small_grid (2 blocks, 512 lanes: a 1 024-slot ring): the launch starts after 512 pushes and renders
    while the host pushes, and pushes wait on the full ring.  staged: the launch counts its jobs per tile and
    vpt_gpu_feed_collect adds the film (copied by the copy engines) and the counts into a host film, then
    clears the device film."""
    import ctypes as C

    import torch

    from volume_path_tracer_amd import capi
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c3", width=96, height=80, spp=24, grid_n=64)
    dens = SynthGrid(1, 64).grid()
    it = Integrator(wl.cfg, dens, None, device=0)
    if mode != "full_grid":
        it.set_tuning(grid_blocks=2)
    staged = mode.startswith("staged")
    L = capi.lib()
    T = wl.cfg.jobs_per_wave()
    rng = np.random.default_rng(3)
    jids = rng.permutation(24 * T)[: 24 * T - 37].astype(np.uint64)  # 37 jobs never pushed
    films = [torch.zeros_like(it.film) for _ in range(2)]
    streams = [C.c_void_p() for _ in range(2)]
    for s in streams:
        capi.check(L.vpt_gpu_stream_create(it.h, C.byref(s)), "stream")
    feeds = []
    halves = np.array_split(jids, 2)
    open_fn = L.vpt_gpu_feed_open_staged if staged else L.vpt_gpu_feed_open
    for k in range(2):
        f = C.c_void_p()
        capi.check(open_fn(it.h, C.c_void_p(films[k].data_ptr()), streams[k], 1000, C.byref(f)), "open")
        feeds.append(f)
    for part in np.array_split(halves[0], 7):
        capi.check(L.vpt_gpu_feed_push(feeds[0], part.ctypes.data_as(C.POINTER(C.c_uint64)), part.size), "push")
    capi.check(L.vpt_gpu_feed_close(feeds[0]), "close")  # the first launch holds the CUs until then
    capi.check(L.vpt_gpu_feed_push(feeds[1], halves[1].ctypes.data_as(C.POINTER(C.c_uint64)), halves[1].size), "push")
    capi.check(L.vpt_gpu_feed_close(feeds[1]), "close")
    host = np.zeros((wl.cfg.height, wl.cfg.width, 4), np.float32)
    for f in feeds:
        if staged:
            capi.check(L.vpt_gpu_feed_collect(f, host.ctypes.data_as(C.POINTER(C.c_float))), "collect")
        else:
            capi.check(L.vpt_gpu_feed_destroy(f), "destroy")
    for s in streams:
        capi.check(L.vpt_gpu_stream_destroy(it.h, s), "stream destroy")
    if staged:
        total = host
        # the collects cleared the device films after copying them out
        assert not films[0].any().item() and not films[1].any().item()
    else:
        total = (films[0] + films[1]).cpu().numpy()
    od = O.OracleGrid(dens, fix_majorants=True)
    ref = np.zeros_like(total)
    # the oracle renders the pushed jobs (contiguous runs of the sorted ids)
    s = np.sort(jids).astype(np.int64)
    breaks = np.flatnonzero(np.diff(s) != 1) + 1
    for run in np.split(s, breaks):
        f, _, _ = O.render_jobs(wl.cfg, od, None, int(run[0]), int(run.size))
        ref += f
    counts = np.bincount((jids % T).astype(np.int64), minlength=T).reshape(wl.cfg.height // 8, wl.cfg.width // 8)
    np.testing.assert_array_equal(total[..., 3], np.kron(counts, np.ones((8, 8))))
    np.testing.assert_allclose(total[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_python_run_snapshots_every_batch():
    """render.run (the Python drop-in) with a progressive-film snapshot after every batch of 7 tokens
    (flush_seconds 0): many copies of the running launch's film and counts added into the host film, then the
    collect -- the film equals the oracle's and every sample is counted once."""
    from volume_path_tracer_amd.render import Integrator, TileProvider, run

    w, h, waves = 40, 24, 3
    wl = workload("c3", width=w, height=h, spp=waves, grid_n=64)
    it = Integrator(wl.cfg, SynthGrid(1, 64).grid(), None, device=0)
    tp = TileProvider(wl.cfg.output_size, waves, wl.cfg.tile_size)
    film = run(wl.cfg, it, tp, batch_jobs=7, flush_seconds=0.0, window=1024)
    np.testing.assert_array_equal(film[..., 3], waves)
    ref = _oracle_film("c3", w, h, waves)
    np.testing.assert_allclose(film[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_python_run_single_pixel():
    """render.run with the reference's single-pixel mode (worker.cpp:113-116): only that pixel gains samples
    and counts -- the counts a staged feed's collect adds on the host follow the same rule as the count
    kernel's."""
    from volume_path_tracer_amd.render import Integrator, TileProvider, run

    w, h, waves = 40, 24, 4
    wl = workload("c3", width=w, height=h, spp=waves, grid_n=64)
    wp = wl.cfg.worker_parameters
    wp.single_pixel_enabled = 1
    wp.single_pixel_coord[0], wp.single_pixel_coord[1] = 13, 9
    dens = SynthGrid(1, 64).grid()
    it = Integrator(wl.cfg, dens, None, device=0)
    tp = TileProvider(wl.cfg.output_size, waves, wl.cfg.tile_size)
    film = run(wl.cfg, it, tp, batch_jobs=11, flush_seconds=0.0)
    want = np.zeros((h, w), np.float32)
    want[9, 13] = waves
    np.testing.assert_array_equal(film[..., 3], want)
    od = O.OracleGrid(dens, fix_majorants=True)
    ref, _, _ = O.render_jobs(wl.cfg, od, None, 0, wl.cfg.jobs_per_wave() * waves)
    np.testing.assert_allclose(film[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_context_waits_refuse_while_a_feed_is_open():
    """while a feed of the context is launched and not closed, the calls that wait for
    the context's launches (vpt_gpu_sync, vpt_gpu_film_clear, vpt_gpu_counters, vpt_gpu_set_tuning) return
    VPT_E_STATE at once instead of waiting for the feed's lanes to give up (30 s) and losing its work.  After
    the close they succeed, and the feed's film holds every pushed job (oracle, exact counts)."""
    import ctypes as C
    import time

    import torch

    from volume_path_tracer_amd import capi
    from volume_path_tracer_amd.render import Integrator

    VPT_E_STATE = 6
    wl = workload("c3", width=64, height=48, spp=16, grid_n=64)
    dens = SynthGrid(1, 64).grid()
    it = Integrator(wl.cfg, dens, None, device=0)
    it.set_tuning(grid_blocks=2)  # 512 lanes: the feed launches once 512 of the 768 jobs are pushed
    L = capi.lib()
    T = wl.cfg.jobs_per_wave()
    film = torch.zeros_like(it.film)
    torch.cuda.synchronize()
    s, f = C.c_void_p(), C.c_void_p()
    capi.check(L.vpt_gpu_stream_create(it.h, C.byref(s)), "stream")
    capi.check(L.vpt_gpu_feed_open(it.h, C.c_void_p(film.data_ptr()), s, 1024, C.byref(f)), "open")
    jids = np.arange(16 * T, dtype=np.uint64)
    capi.check(L.vpt_gpu_feed_push(f, jids.ctypes.data_as(C.POINTER(C.c_uint64)), jids.size), "push")  # launched
    t0 = time.monotonic()
    assert L.vpt_gpu_sync(it.h) == VPT_E_STATE
    assert L.vpt_gpu_film_clear(it.h) == VPT_E_STATE
    assert L.vpt_gpu_set_tuning(it.h, 6, 8, 0, 36, 4) == VPT_E_STATE
    assert time.monotonic() - t0 < 5.0
    capi.check(L.vpt_gpu_feed_close(f), "close")
    capi.check(L.vpt_gpu_feed_destroy(f), "destroy")
    capi.check(L.vpt_gpu_sync(it.h), "sync after the close")
    capi.check(L.vpt_gpu_stream_destroy(it.h, s), "stream destroy")
    out = film.cpu().numpy()
    np.testing.assert_array_equal(out[..., 3], 16)
    ref = _oracle_film("c3", 64, 48, 16)
    np.testing.assert_allclose(out[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_stale_waiting_word_is_overwritten_while_lanes_wait():
    """the backlog estimate reads 0 once the lanes wait, from the "waiting" word a wavefront
    stores when it runs out of published jobs -- but an older count's posted write may land after a newer one.
    Waiting wavefronts now store the count again every ~5 ms, and the host reads hints that have not moved for
    10 ms as an empty backlog.  Here a launch's lanes have taken every pushed job and wait; a stale "waiting" word
    and stale hints are planted (vpt_gpu_feed_debug): the lanes overwrite the word within 50 ms and the estimate
    reads 0, so a pusher never waits on it; then more pushes render and the film is exact."""
    import ctypes as C
    import time

    import torch

    from volume_path_tracer_amd import capi
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c3", width=64, height=48, spp=20, grid_n=64)
    it = Integrator(wl.cfg, SynthGrid(1, 64).grid(), None, device=0)
    it.set_tuning(grid_blocks=2)  # 512 lanes: launched once 512 jobs are pushed
    L = capi.lib()
    T = wl.cfg.jobs_per_wave()
    film = torch.zeros_like(it.film)
    torch.cuda.synchronize()
    s, f = C.c_void_p(), C.c_void_p()
    capi.check(L.vpt_gpu_stream_create(it.h, C.byref(s)), "stream")
    capi.check(L.vpt_gpu_feed_open(it.h, C.c_void_p(film.data_ptr()), s, 2048, C.byref(f)), "open")
    jids = np.arange(16 * T, dtype=np.uint64)
    capi.check(L.vpt_gpu_feed_push(f, jids.ctypes.data_as(C.POINTER(C.c_uint64)), jids.size), "push")
    v, b = C.c_uint64(), C.c_uint64()
    t0 = time.monotonic()
    while True:  # the lanes take every job, then wait
        capi.check(L.vpt_gpu_feed_debug(f, 0, C.byref(v)), "debug")
        if v.value >= jids.size or time.monotonic() - t0 > 10:
            break
        time.sleep(0.001)
    assert v.value >= jids.size, v.value
    v.value = 3  # an old count landing last
    capi.check(L.vpt_gpu_feed_debug(f, 1, C.byref(v)), "plant waiting")
    v.value = 5
    capi.check(L.vpt_gpu_feed_debug(f, 2, C.byref(v)), "plant hints")
    t0 = time.monotonic()
    while True:
        capi.check(L.vpt_gpu_feed_debug(f, 0, C.byref(v)), "debug")
        if v.value >= jids.size or time.monotonic() - t0 > 1.0:
            break
        time.sleep(0.0005)
    refresh_ms = (time.monotonic() - t0) * 1e3
    print(f"waiting word rewritten after {refresh_ms:.1f} ms")
    assert v.value >= jids.size and refresh_ms < 50, (v.value, refresh_ms)
    capi.check(L.vpt_gpu_feed_backlog(f, C.byref(b)), "backlog")
    assert b.value == 0, b.value
    more = np.arange(16 * T, 20 * T, dtype=np.uint64)
    capi.check(L.vpt_gpu_feed_push(f, more.ctypes.data_as(C.POINTER(C.c_uint64)), more.size), "push more")
    capi.check(L.vpt_gpu_feed_close(f), "close")
    capi.check(L.vpt_gpu_feed_destroy(f), "destroy")
    capi.check(L.vpt_gpu_stream_destroy(it.h, s), "stream destroy")
    out = film.cpu().numpy()
    np.testing.assert_array_equal(out[..., 3], 20)
    np.testing.assert_allclose(out[..., :3], _oracle_film("c3", 64, 48, 20)[..., :3], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_staged_feed_snapshots_add_up_to_the_film():
    """vpt_gpu_feed_snapshot while the launch renders (the drop-in's progressive film): several snapshots of a
    running staged feed, then the collect.  The host film's sample counts never exceed the jobs pushed and end
    exact; its radiance equals the oracle's (the snapshots' additions telescope to the launch's film)."""
    import ctypes as C

    import torch

    from volume_path_tracer_amd import capi
    from volume_path_tracer_amd.render import Integrator

    w, h, waves = 96, 64, 48
    wl = workload("c3", width=w, height=h, spp=waves, grid_n=64)
    dens = SynthGrid(1, 64).grid()
    it = Integrator(wl.cfg, dens, None, device=0)
    it.set_tuning(grid_blocks=4)  # 1 024 lanes: the launch renders while the host pushes
    L = capi.lib()
    T = wl.cfg.jobs_per_wave()
    capi.check(L.vpt_gpu_feed_prepare(it.h, 0, 1), "prepare")
    s, f = C.c_void_p(), C.c_void_p()
    capi.check(L.vpt_gpu_stream_create(it.h, C.byref(s)), "stream")
    torch.cuda.synchronize()
    capi.check(L.vpt_gpu_feed_open_staged(it.h, C.c_void_p(it.film.data_ptr()), s, 0, C.byref(f)), "open")
    host = np.zeros((h, w, 4), np.float32)
    hp = host.ctypes.data_as(C.POINTER(C.c_float))
    seen = []
    for wave in range(waves):
        jids = np.arange(wave * T, (wave + 1) * T, dtype=np.uint64)
        capi.check(L.vpt_gpu_feed_push(f, jids.ctypes.data_as(C.POINTER(C.c_uint64)), jids.size), "push")
        b = C.c_uint64()
        capi.check(L.vpt_gpu_feed_backlog(f, C.byref(b)), "backlog")
        assert b.value <= (wave + 1) * T
        if wave % 6 == 5:
            capi.check(L.vpt_gpu_feed_snapshot(f, hp), "snapshot")
            assert (host[..., 3] <= wave + 1).all()
            seen.append(float(host[..., 3].mean()))
    capi.check(L.vpt_gpu_feed_collect(f, hp), "collect")
    capi.check(L.vpt_gpu_stream_destroy(it.h, s), "stream destroy")
    assert all(b >= a for a, b in zip(seen, seen[1:])), seen
    np.testing.assert_array_equal(host[..., 3], waves)
    ref = _oracle_film("c3", w, h, waves)
    np.testing.assert_allclose(host[..., :3], ref[..., :3], rtol=1e-5, atol=1e-6)
    # the collect left the feed's film zero
    assert not it.film.any().item()


@pytest.mark.gpu
def test_bind_thread_near_binds_to_the_gpus_node():
    """vpt_gpu_bind_thread_near: a thread -- here one whose own CPU set was narrowed to a single CPU, as a
    thread inherits its creator's -- ends up on the CPUs of the device's NUMA node that the process may use
    (the node from sysfs, the process's set), or is left as it was when the node is unknown."""
    import ctypes as C
    import os
    import threading

    from volume_path_tracer_amd import capi
    from volume_path_tracer_amd.render import Integrator

    wl = workload("c3", width=32, height=32, spp=1, grid_n=64)
    it = Integrator(wl.cfg, SynthGrid(1, 64).grid(), None, device=0)
    proc = os.sched_getaffinity(0)
    out = {}

    def body():
        os.sched_setaffinity(0, {min(proc)})
        node = C.c_int(-2)
        out["rc"] = capi.lib().vpt_gpu_bind_thread_near(it.h, C.byref(node))
        out["node"], out["cpus"] = node.value, os.sched_getaffinity(0)

    t = threading.Thread(target=body)
    t.start()
    t.join()
    assert out["rc"] == 0
    if out["node"] < 0:
        assert out["cpus"] == {min(proc)}
        return
    text = Path(f"/sys/devices/system/node/node{out['node']}/cpulist").read_text().strip()
    node_cpus = set()
    for part in text.split(","):
        a, _, b = part.partition("-")
        node_cpus.update(range(int(a), int(b or a) + 1))
    assert out["cpus"] == node_cpus & proc, (out["node"], sorted(out["cpus"])[:8])
