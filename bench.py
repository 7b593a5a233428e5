#!/usr/bin/env python3
"""Benchmark: Msamples/s of the volumetric path-tracing integrator on BASELINE.json's headline
workload (configs[2]: wdas_cloud.json at 1920x1080, 256 spp, one MI355X), on the synthetic 512^3
cloud stand-in (the reference's wdas_cloud.nvdb is not available).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]

One step = one full frame (every wave of the configuration) rendered into a zeroed film on every
rank, plus — for N > 1 — the RCCL sum of the films over xGMI.

Multi-GPU.  `--gpus N` runs N ranks, one per GPU: under torchrun (WORLD_SIZE must equal N), or, when
WORLD_SIZE is unset, by starting torch.distributed.run itself before anything touches the GPU.
  * default `--mode weak` (the driver's SCALE runs): every rank renders its own block of the C3
    frame's 256 waves (rank r: waves r*256+1 .. (r+1)*256), so N = 1 is exactly BENCH's C3 line and
    the per-GPU work is fixed;
  * for N > 1 the line also carries `scaling_strong`: the C3 frame (256 waves) and the C5 frame
    (BASELINE.json configs[4], 3840x2160 at 1024 spp) each dealt across the N ranks and timed the same
    way (barrier + synchronize, max over ranks, film all-reduce inside the step): the strong scaling
    that north_star's ">= 6x at 8 GPUs" asks about (`--strong-configs`, '' to skip); and the C3 frame in
    the throughput mode ("c3:pixel": per-pixel streams, reported separately, never the headline);
  * `--config c5 --mode strong --gpus 8` makes the C5 frame the main measurement.

The JSON line also carries:
  roofline      the integrator kernel's algorithmic bytes per launch (SURVEY §8d:
                32*stencils + 8*dda_steps + 32*temp_stencils + 32*samples, from the kernel's own
                event counters) / its average launch time (HIP events on the launch stream), against
                the 8 TB/s HBM peak; `traffic` = PMC-measured HBM bytes per launch from the newest
                committed profiles/<round>_<config>_pmc.json (a builder rocprofv3 --pmc pass, named in
                `traffic_source`), else null.
  cpu_baseline  the CPU oracle (headless restatement of the reference worker pool, main.cpp:62-87)
                timed on this host's cores on a bounded sample (whole waves of the same frame).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def baseline_metric() -> str:
    """BASELINE.json's headline metric string (the C3 workload; other configs say theirs in config)."""
    try:
        return json.loads((ROOT / "BASELINE.json").read_text())["metric"]
    except Exception:
        return "Msamples/s (whole node) + achieved HBM GB/s, wdas_cloud 1920\u00d71080"


def algorithmic_bytes(c: dict) -> int:
    return 32 * c["stencils"] + 8 * c["dda_steps"] + 32 * c["temp_stencils"] + 32 * c["samples"]


def host_cpu_info() -> dict:
    """The host's CPUs as this process sees them: nproc, the affinity mask, the cgroup CPU quota
    (cpu.max, when limited) and the model name."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except Exception:
        info["affinity"] = os.cpu_count()
    info["cgroup_cpus"] = None
    try:
        quota, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if quota != "max":
            info["cgroup_cpus"] = round(int(quota) / int(period), 2)
    except Exception:
        pass
    info["cpu_model"] = None
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                info["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return info


def cpu_baseline(wl, dens, temp, budget_s: float = 15.0, runs: int = 3):
    """The reference worker pool (main.cpp:62-87, restated headless in the oracle: one std::thread per
    core calling run() over a TileProvider) on every CPU this process may use, over the
    DISTINCT waves 1..k of the workload's frame (k sized so that `runs` runs take ~budget_s);
    the value is the median of the runs' Msamples/s."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O

    info = host_cpu_info()
    # every CPU this process may run on: the affinity mask, capped by the cgroup CPU quota (threads
    # beyond the quota only time-slice; the GPU box grants a 1-GPU job 16 of its 256 CPUs)
    threads = max(1, info["affinity"] or 1)
    if info["cgroup_cpus"]:
        threads = max(1, min(threads, int(info["cgroup_cpus"] + 0.5)))
    od = O.OracleGrid(dens, fix_majorants=True)
    ot = O.OracleGrid(temp, fix_majorants=False) if temp is not None else None
    cfg = wl.cfg.copy()
    per_wave = cfg.width * cfg.height
    _, ms1, _ = O.render_pool(cfg, od, ot, 1, threads)  # calibration: wave 1
    k = int(max(1, min(wl.spp, budget_s / runs / max(ms1 / 1e3, 1e-3))))
    rates, secs = [], []
    film = None
    for _ in range(runs):
        film, ms, _ = O.render_pool(cfg, od, ot, k, threads)
        rates.append(k * per_wave / (ms / 1e3) / 1e6)
        secs.append(ms / 1e3)
    rates.sort()
    med = rates[len(rates) // 2]
    node = info["nproc"] or threads
    return {"value": round(med, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"waves 1..{k} of {cfg.width}x{cfg.height} ({k * per_wave} samples) per run, median of {runs} "
                      f"runs ({', '.join(f'{r:.3f}' for r in rates)} Msamples/s, {sum(secs):.1f} s), oracle worker "
                      f"pool (main.cpp:62-87 restated), {threads} threads",
            "spread": round((rates[-1] - rates[0]) / med, 4),
            "per_thread": round(med / threads, 5), "host": info,
            # not measured: the per-thread rate times every hardware thread of the node (the job is granted
            # `cores` of them), an upper bound that ignores SMT and memory contention
            "node_extrapolated": {"threads": node, "value": round(med / threads * node, 3), "unit": "Msamples/s",
                                  "kind": "linear extrapolation of per_thread, not a measurement"}}, film, k


def film_parity(wl, dens, temp, ref_film, waves: int, device: int) -> dict:
    """north_star's parity criterion on the bench's own frame: the production kernel renders the waves the CPU
    baseline just rendered with the oracle's worker pool (waves 1..k, the same jobs and PCG streams), and the
    per-pixel radiance (film XYZ / sample count) is compared -- RMSE over every pixel and channel against the
    stated bound of 1e-4, the largest difference, and the sample counts (which must be equal).  With the ordered
    film (the default, vpt_gpu_set_film_order) the GPU adds each pixel's samples in wave order, the oracle's
    order, so the two films are compared bit for bit too (`bit_identical`, `pixels_differing`)."""
    import numpy as np
    import torch

    from volume_path_tracer_amd.render import Integrator

    it = Integrator(wl.cfg, dens, temp, device=device)
    it.render_waves(1, waves)
    torch.cuda.synchronize()
    gpu = it.film_host()
    film_mode = it.film_order_info()
    del it
    differ = int((gpu.view(np.uint32) != ref_film.view(np.uint32)).any(axis=-1).sum())
    counts_equal = bool(np.array_equal(gpu[..., 3], ref_film[..., 3]))
    n = np.maximum(ref_film[..., 3:4].astype(np.float64), 1.0)
    lg, lr = gpu[..., :3].astype(np.float64) / n, ref_film[..., :3].astype(np.float64) / n
    rmse = float(np.sqrt(np.mean((lg - lr) ** 2)))
    return {"waves": waves, "pixels": int(lg.shape[0] * lg.shape[1]), "counts_equal": counts_equal,
            "rmse_per_pixel": rmse, "max_abs_diff": float(np.abs(lg - lr).max()),
            "mean_radiance": float(np.abs(lr).mean()), "bound": 1e-4, "ok": counts_equal and rmse < 1e-4,
            "bit_identical": differ == 0, "pixels_differing": differ,
            "film_order": "ordered (wave order)" if film_mode["mode"] == 1 else "atomic",
            "vs": "oracle worker pool (tests/oracle_lib.py render_pool), same waves and seeds"}


HARNESS = ROOT / "tests" / "native" / "build" / "run_gpu_harness"


def dropin_frames(wl, frames: int = 3, timeout_s: int = 300):
    """The reference-API path, timed: main.cpp:46-87 made headless -- the restated
    TileProvider and one worker thread calling vpt_gpu::drain (include/vpt_run.hpp: one staged feed, the
    pusher and film threads, the 0.2-s progressive film, and run()'s ordered frame: the film in wave order at the
    end, DrainOptions::ordered_frame) -- through tests/native/run_gpu_harness, on this
    config's frame: `frames` frames on one context (setup -- grid upload, tile costs, the feed's memory --
    outside the timed drains, as the harness and run_checked do it) after one untimed frame.  The median of the
    frames is the record's ms_per_frame.  Then the provider alone (mode=tokens: one
    thread taking every token of the frame), the drop-in's host-side floor.  A child process, started before
    this process touches the GPU.  None for C5 (one GPU's frame of BASELINE's 8-GPU configuration)."""
    import subprocess
    import tempfile

    if wl.name not in ("c1", "c2", "c3", "c4") or not HARNESS.exists():
        return None
    scene = ROOT / "volume_path_tracer_amd" / "scenes" / ("fire.json" if wl.temperature else "wdas_cloud.json")
    W, H, spp = wl.cfg.width, wl.cfg.height, wl.spp
    with tempfile.TemporaryDirectory() as tmp:
        if wl.name == "c2":  # the constant cube: wdas_cloud.json with C2's medium (scenes.workload), camera at 300
            doc = json.loads(scene.read_text())
            v = wl.cfg.volume_parameters
            vp = doc["volume_parameters"]
            vp.update(sigma_s=v.sigma_s, sigma_a=v.sigma_a, henyey_greenstein_g=v.henyey_greenstein_g, le_scale=v.le_scale)
            scene = Path(tmp) / "c2.json"
            scene.write_text(json.dumps(doc))
        base = [str(HARNESS), f"config={scene}", f"w={W}", f"h={H}", f"waves={spp}", f"grid_n={wl.grid_n}",
                f"kind={wl.density_kind}", f"dist={-wl.cfg.camera_parameters.position[2]:g}", "threads=1", "batch=4096",
                f"temperature={1 if wl.temperature else 0}", "ordered=1"]
        try:
            r = subprocess.run(base + [f"out={tmp}/film.f32", f"frames={frames}", "warmup=1"], capture_output=True,
                               text=True, timeout=timeout_s)
        except subprocess.TimeoutExpired:  # (the bench line still prints; the record says what happened)
            log(f"bench: drop-in harness timed out after {timeout_s} s")
            return {"error": f"timeout {timeout_s} s"}
        if r.returncode != 0:
            log(f"bench: drop-in harness failed ({r.returncode}): {r.stderr[-500:]}")
            return {"error": r.returncode}
        film = __import__("numpy").fromfile(f"{tmp}/film.f32", "float32").reshape(H, W, 4)
        counts_ok = bool((film[..., 3] == spp).all())
        try:
            t = subprocess.run(base + [f"out={tmp}/x", "mode=tokens"], capture_output=True, text=True, timeout=60)
        except subprocess.TimeoutExpired:
            t = None
        first = first_call(wl, base, tmp, timeout_s)
    ms = [float(l.split()[-1]) for l in r.stdout.splitlines() if "render_ms" in l]
    if not ms:  # (a harness that printed no frame time is recorded, not fatal)
        return {"error": "no render_ms lines", "stdout_tail": r.stdout[-500:]}
    med = sorted(ms)[len(ms) // 2]
    rec = {"path": "vpt_gpu::drain (include/vpt_run.hpp) behind the restated TileProvider, main.cpp:46-87 headless "
                   "(tests/native/run_gpu_harness), 1 worker thread, 0.2-s progressive film, ordered frame (as run())",
           "_film": film,
           "workload": f"{wl.name}: {W}x{H}, {spp} spp", "frames": len(ms), "warmup_frames": 1, "ms_frames": ms,
           "ms_per_frame": med,
           "value": round(W * H * spp / (med / 1e3) / 1e6, 3), "unit": "Msamples/s", "film_counts_exact": counts_ok}
    for line in (t.stdout.splitlines() if t is not None else []):
        if "tokens_ms" in line:  # "tokens_ms 125.5, 8294400 tokens, 66.1 M tokens/s, 1 threads"
            parts = line.replace(",", "").split()
            rec["provider_alone_ms"] = float(parts[parts.index("tokens_ms") + 1])
            rec["provider_alone_Mtokens_per_s"] = float(parts[parts.index("M") - 1])
    rec["first_call"] = first
    return rec


def first_call(wl, base, tmp, timeout_s):
    """What a reference caller's run() costs: main.cpp renders one frame per process and times the
    whole vpt::run call ("Rendering complete in N ms", main.cpp:65-84).  A fresh child process runs
    vpt_gpu::run (include/vpt_run.hpp) with the reference's own argument types -- the volume as NanoGrid<float>
    bytes, the seed private to the RandomNumberGenerator -- from the scene's num_workers threads (the first
    drives the GPU, the others return), and reports the call's phases: the HIP runtime's start, the first
    batch of tokens, the seed recovery (one GPU launch over 2^32 candidates), reading the NanoGrids, the
    context (flatten + leaf-majorant fix, upload, the rest, the tile-cost pass), and the frame."""
    import subprocess

    from volume_path_tracer_amd import nvdb
    from volume_path_tracer_amd.scenes import SynthGrid

    t0 = time.time()
    dg = SynthGrid(wl.density_kind, wl.grid_n)
    (Path(tmp) / "density.grid").write_bytes(nvdb.buffer_from_grid(dg.grid(copy=False), "density"))
    extra = [f"gridbuf={tmp}/density.grid"]
    if wl.temperature:
        tg = SynthGrid(2, wl.grid_n)
        (Path(tmp) / "temperature.grid").write_bytes(nvdb.buffer_from_grid(tg.grid(copy=False), "temperature"))
        extra.append(f"tempbuf={tmp}/temperature.grid")
    prep_s = time.time() - t0
    args = [a for a in base if not a.startswith("threads=")] + extra + [f"out={tmp}/first.f32", "mode=run",
                                                                         f"threads={wl.cfg.num_workers or 1}"]
    try:
        r = subprocess.run(args, capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"error": f"timeout {timeout_s} s"}
    if r.returncode != 0:
        return {"error": r.returncode, "stderr_tail": r.stderr[-500:]}
    rec = {"path": "vpt_gpu::run (include/vpt_run.hpp) in a fresh process, main.cpp:63-68's call with the reference's "
                   "types (tests/native/run_gpu_harness mode=run): NanoGrid<float> bytes, private seed",
           "worker_threads": wl.cfg.num_workers, "grid_bytes_written_s": round(prep_s, 2)}
    for line in r.stdout.splitlines():
        if "phases" in line:
            for kv in line.split("phases", 1)[1].split():
                k, _, v = kv.partition("=")
                rec[k] = float(v) if "." in v else int(v)
    W, H = wl.cfg.width, wl.cfg.height
    film = __import__("numpy").fromfile(f"{tmp}/first.f32", "float32").reshape(H, W, 4)
    rec["film_counts_exact"] = bool((film[..., 3] == wl.spp).all())
    rec["note"] = ("total_ms = the whole run() call as main.cpp times it; the grid load itself (NanoVDB file read, "
                   "Volume ctor) happens before it in main.cpp:40-41 and is not in it. hip_ms + seed_ms run on a helper "
                   "thread beside nanogrid_ms; wait_ms is the wait for it after the read. contexts_ms = the contexts "
                   "(upload_ms, ctx_rest_ms) + feeds_ms (the feed's pinned memory and tile_costs_ms); flatten_ms runs "
                   "beside the helper too. The host copies of the flattened grids are kept until the next run() or the "
                   "process's exit, as the reference's Volume keeps its grids")
    return rec


def spawn_ranks(args) -> int:
    """--gpus N without torchrun's environment: start N fresh ranks (this process has not touched the
    GPU) through torch.distributed.run on 127.0.0.1, and return their exit code."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve()), *sys.argv[1:]]
    log(f"bench: starting {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd).returncode


def newest_profile(pattern: str, match=lambda j: True):
    """(json, 'profiles/<name>') of the newest committed profiles/<pattern> that matches, or (None, None)."""
    for pf in sorted((ROOT / "profiles").glob(pattern), reverse=True):
        try:
            j = json.loads(pf.read_text())
        except Exception:
            continue
        if match(j):
            return j, f"profiles/{pf.name}"
    return None, None


def request_roofline(config: str, samples_per_launch: float, avg_launch_s: float, cus: int) -> dict:
    """The binding limit of the walk: L1->L2 read requests per second per CU against the
    measured ceiling of divergent 4-byte per-lane gathers from an L2-resident table
    (tools/ubench/gather.hip).  Requests per sample come from the newest committed rocprofv3 counter
    pass of this config (tools/kernel_counters.sh) -- builder measurements, named in the line --
    times this run's samples per launch over this run's average launch time."""
    cnt, cnt_src = newest_profile("*_counters.json", lambda j: j.get("config") == config and not j.get("bench_args") and
                                  j.get("derived", {}).get("l1_to_l2_requests_per_sample"))
    ceil, ceil_src = newest_profile("*_gather_ceiling.json")
    if not cnt or not ceil:
        return {"request_frac": None}
    achieved = cnt["derived"]["l1_to_l2_requests_per_sample"] * samples_per_launch / avg_launch_s / cus
    peak = ceil["ceiling_l1_to_l2_requests_per_s_per_cu"]
    return {"request_frac": round(achieved / peak, 4),
            "request_achieved_per_s_per_cu": round(achieved, 1), "request_peak_per_s_per_cu": round(peak, 1),
            "request_sources": [cnt_src, ceil_src]}


POOL_BYTES_PER_LEAF = 9216  # the stencil pool: per leaf 8 x 8 voxel rows of 9 2x2 squares (include/vpt_gpu.h)
STRADDLE = 1.125            # L1->L2 requests per stencil piece: 1 pair in 8 straddles a 128-B line


def interp_loglog(points, x):
    """Log-log interpolation of [(x, y)] at x (clamped to the measured range)."""
    import math

    pts = sorted(points)
    if x <= pts[0][0]:
        return pts[0][1]
    if x >= pts[-1][0]:
        return pts[-1][1]
    for (x0, y0), (x1, y1) in zip(pts, pts[1:]):
        if x0 <= x <= x1:
            f = (math.log(x) - math.log(x0)) / (math.log(x1) - math.log(x0))
            return math.exp(math.log(y0) + f * (math.log(y1) - math.log(y0)))
    return pts[-1][1]


def pipe_roofline(config: str, samples_per_s_per_cu: float, stencil_entries_per_sample: float, pool_mib: float) -> dict:
    """The vector-memory pipeline as two request classes: stencil pieces gathered from the
    stencil pool (L2 misses: ~every one) at the measured rate of random 32-B gathers from a table of the
    pool's size (tools/ubench/gather pool), and every other L1->L2 request (walk words, cell entries: L2
    hits) at the measured L2-resident 4-B gather ceiling.  pipe_frac = the sum of the two classes' shares
    of the pipeline's time, from this run's rate and stencil count, the newest committed counter pass's
    requests per sample and the two ceiling files (all named in pipe_sources)."""
    cnt, cnt_src = newest_profile("*_counters.json", lambda j: j.get("config") == config and not j.get("bench_args") and
                                  j.get("derived", {}).get("l1_to_l2_requests_per_sample"))
    ceil, ceil_src = newest_profile("*_gather_ceiling.json")
    pool, pool_src = newest_profile("*_pool_ceiling.json")
    if not cnt or not ceil or not pool:
        return {"pipe_frac": None}
    stencil_ceiling = interp_loglog([(p["table_mib"], p["entries_per_s_per_cu"]) for p in pool["points"]], pool_mib)
    other = max(0.0, cnt["derived"]["l1_to_l2_requests_per_sample"] - STRADDLE * stencil_entries_per_sample)
    st = stencil_entries_per_sample * samples_per_s_per_cu / stencil_ceiling
    ot = other * samples_per_s_per_cu / ceil["ceiling_l1_to_l2_requests_per_s_per_cu"]
    return {"pipe_frac": round(st + ot, 4), "pipe_stencil_share": round(st, 4), "pipe_other_share": round(ot, 4),
            "pipe_pool_mib": round(pool_mib, 1), "pipe_sources": [cnt_src, ceil_src, pool_src]}


def mix_roofline(config: str, spp: int, avg_launch_s: float, frame_samples: float, samples_per_launch: float) -> dict:
    """The launch's memory work alone, measured: the newest committed profiles/*_<config>_mix_ceiling.json
    (tools/ubench/gather mix: the config's per-sample request mix -- walk-class 4-B gathers from an L2-resident
    table, 32-B pool gathers, both dependent chains -- chased at the kernel's occupancy with half the lanes
    active, no arithmetic) gives the frame's memory-only time; mix_frac = that time / this launch's time, scaled
    to this launch's samples.  Unlike pipe_frac (two classes priced apart and added) one chase prices the mix
    jointly (r05: C3 0.51, C4 0.28 -- the kernels are not at their memory ceiling)."""
    mj, src = newest_profile("*_mix_ceiling.json", lambda j: j.get("config") == config and j.get("spp") == spp)
    if not mj or not frame_samples:  # (measured for the full launches, C3 / C4; C1 / C2 are latency-bound)
        return {}
    mix_ms = mj["frame_ms"] * samples_per_launch / frame_samples
    return {"mix_frac": round(mix_ms / (avg_launch_s * 1e3), 4), "mix_ms_per_launch": round(mix_ms, 2),
            "mix_source": src}


def init_rank(args, env=None):
    """(rank, world, device, scalar device) of this process.  One process per GPU: device LOCAL_RANK
    (device 0 for --one-device, the one-GPU multi-process tests).  For world > 1 the process group is
    RCCL over xGMI ("nccl", bound to the rank's device with device_id) or gloo (CPU-side tests);
    scalars (timings, sample counts) travel on the device with RCCL, through the host with gloo."""
    import torch
    import torch.distributed as dist

    env = os.environ if env is None else env
    world = int(env.get("WORLD_SIZE", "1"))
    rank = int(env.get("RANK", "0"))
    local = int(env.get("LOCAL_RANK", "0"))
    dev_index = 0 if (world == 1 or args.one_device) else local
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        env.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    sdev = dev if args.backend == "nccl" else torch.device("cpu")
    return rank, world, dev, sdev


def max_over_ranks(x: float, world: int, sdev) -> float:
    import torch
    import torch.distributed as dist

    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=sdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: int, world: int, sdev) -> int:
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device=sdev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def timed_frames(it, rank, world, spp, mode, steps, warmup, stream, launch_ms=None, reduce=True):
    """`warmup` untimed then `steps` timed frames (this rank's share of the spp waves, then the film
    all-reduce), bracketed by a barrier and torch.cuda.synchronize() on both sides; returns this rank's
    timed region (seconds; the caller takes the MAX over ranks).  launch_ms collects HIP-event pairs
    around each frame's kernel launches (on the launch stream).  world = 1 with reduce=False times one
    rank alone (no collective: the other ranks are not in the step)."""
    import torch
    import torch.distributed as dist

    from volume_path_tracer_amd import distributed as D

    def step(timed: bool):
        it.film.zero_()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(stream)  # the kernel runs on this stream: the events bracket exactly its launches
        D.render_rank(it, rank, world, spp, mode, stream=stream)
        ev1.record(stream)
        if timed and launch_ms is not None:
            launch_ms.append((ev0, ev1))
        if reduce:
            D.reduce_film(it.film)

    for _ in range(warmup):
        step(False)
    torch.cuda.synchronize()
    it.counters(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t_start


ALONE_BIG_SAMPLES = 1e9  # frames this large (C5: 8.5e9 samples, ~5 s on one GPU) are timed alone at 1 + 1 frames


def strong_scaling(configs, dens, rank, world, dev, sdev, steps, warmup, stream):
    """For N > 1: each config's whole frame (its spp waves) dealt across the N ranks (distributed
    "strong" ranges), timed like the main loop -- the work the north_star's "scaling at 8 GPUs" means
    (C3: the headline frame; C5: BASELINE's 8-GPU configuration, 3840x2160 at 1024 spp, on which the
    ">= 6x at 8 GPUs" target is judged).  Then the same whole frame on rank 0's GPU alone, timed the same
    way while the other ranks wait at a barrier (1 warmup + 1 step for frames of >= 1e9 samples), so the
    record carries its own speedup_vs_1gpu = t(1 GPU) / t(N GPUs) and efficiency = speedup / N."""
    import torch.distributed as dist

    from volume_path_tracer_amd import capi
    from volume_path_tracer_amd import distributed as D
    from volume_path_tracer_amd.render import Integrator
    from volume_path_tracer_amd.scenes import workload

    out = {}
    for name in configs:
        base, _, mode = name.partition(":")  # "c3:pixel" = the throughput mode's per-pixel streams
        if mode not in ("", "pixel"):
            raise ValueError(f"--strong-configs: unknown mode in {name}")
        wl = workload(base)
        if wl.temperature or wl.density_kind != 1 or wl.grid_n != 512:
            raise ValueError(f"--strong-configs: {name} does not share the 512^3 cloud stand-in")
        it = Integrator(wl.cfg, dens, None, device=dev.index)
        if mode == "pixel":
            it.set_rng_mode(capi.VPT_RNG_PIXEL)
        elapsed = max_over_ranks(timed_frames(it, rank, world, wl.spp, "strong", steps, warmup, stream), world, sdev)
        samples = sum_over_ranks(it.counters()["samples"], world, sdev)
        film = it.film_host()
        assert (film[..., 3] == D.total_samples_per_pixel(world, wl.spp, "strong")).all(), "sample-count channel mismatch"
        assert samples == wl.cfg.width * wl.cfg.height * wl.spp * steps, samples
        frame = wl.cfg.width * wl.cfg.height * wl.spp
        s1, w1 = (1, 1) if frame >= ALONE_BIG_SAMPLES else (steps, warmup)
        dist.barrier()
        alone = None
        if rank == 0:
            alone = timed_frames(it, 0, 1, wl.spp, "strong", s1, w1, stream, reduce=False)
            film = it.film_host()
            assert (film[..., 3] == wl.spp).all(), "sample-count channel mismatch (1-GPU frame)"
        dist.barrier()
        rec = {"workload": f"{base}: {wl.cfg.width}x{wl.cfg.height}, {wl.spp} spp per image, dealt over {world} GPUs"
                           + (" (throughput mode: per-pixel streams, not the reference's samples)" if mode else ""),
               "ms_per_step": round(elapsed / steps * 1e3, 3), "value": round(samples / elapsed / 1e6, 3),
               "unit": "Msamples/s", "steps": steps, "warmup": warmup}
        if alone is not None:
            t1, tn = alone / s1, elapsed / steps
            rec.update(one_gpu_ms_per_step=round(t1 * 1e3, 3), one_gpu_steps=s1, one_gpu_warmup=w1,
                       speedup_vs_1gpu=round(t1 / tn, 3), efficiency=round(t1 / tn / world, 4))
        out[name] = rec
        del it
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--spp", type=int, default=None, help="override waves per step (default: the config's)")
    ap.add_argument("--grid-n", type=int, default=None, help="experiments: override the stand-in grid's size n^3")
    ap.add_argument("--mode", choices=["weak", "strong"], default="weak",
                    help="weak: each rank renders its own spp waves; strong: the spp waves are dealt across ranks")
    ap.add_argument("--strong-configs", default="c3,c5,c3:pixel",
                    help="N > 1: configs whose whole frame is also timed dealt across the ranks ('' = none; "
                         "':pixel' = in the throughput mode)")
    ap.add_argument("--rng-mode", choices=["reference", "pixel"], default="reference",
                    help="pixel = throughput mode (per-pixel streams; not the reference's samples)")
    ap.add_argument("--latency-kernel", choices=["auto", "off", "on", "gated"], default="auto",
                    help="the latency kernel (cold lane state in VGPRs): auto = latency-bound launches (C1, latency "
                         "gates) and partly filled ones (C2, small shares; the context's gates); off never; on / gated "
                         "force it with the latency / the context's gates on partly filled launches (A/B runs)")
    ap.add_argument("--compaction", type=int, default=None,
                    help="live-path compaction period on partly filled latency launches (A/B runs; default: the "
                         "library's, off)")
    ap.add_argument("--film-order", choices=["ordered", "atomic"], default="ordered",
                    help="ordered (default): each pixel's samples added in wave order, the reference's film bit for bit "
                         "(vpt_gpu_set_film_order); atomic: fp32 atomics in completion order (A/B runs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the reference-API (drop-in) frame timing")
    ap.add_argument("--dropin-frames", type=int, default=3)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-baseline work (3 runs)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI)")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on device 0 (multi-process tests on a one-GPU box)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}: launch with --nproc-per-node equal to --gpus")
        sys.exit(2)

    import torch
    import torch.distributed as dist

    dropin = None
    # (not under rocprofv3: its preloaded library has initialised the GPU in this process, which then must not
    # start another program)
    profiled = any(k.startswith("ROCPROF") for k in os.environ)
    if (world == 1 and not args.no_dropin and not profiled and args.rng_mode == "reference" and args.spp is None
            and args.grid_n is None):
        # the drop-in runs in a child process, before this one touches the GPU
        from volume_path_tracer_amd.scenes import workload as _workload

        t0 = time.time()
        dropin = dropin_frames(_workload(args.config), args.dropin_frames)
        log(f"bench: drop-in frames in {time.time() - t0:.1f}s: "
            f"{ {k: v for k, v in dropin.items() if k != '_film'} if isinstance(dropin, dict) else dropin}")

    rank, world, dev, sdev = init_rank(args)

    from volume_path_tracer_amd import distributed as D
    from volume_path_tracer_amd.render import Integrator
    from volume_path_tracer_amd.scenes import SynthGrid, workload

    wl = workload(args.config, spp=args.spp, grid_n=args.grid_n)
    t0 = time.time()
    dg = SynthGrid(wl.density_kind, wl.grid_n)
    tg = SynthGrid(2, wl.grid_n) if wl.temperature else None
    dens, temp = dg.grid(copy=False), (tg.grid(copy=False) if tg else None)
    it = Integrator(wl.cfg, dens, temp, device=dev.index)
    if args.rng_mode == "pixel":
        from volume_path_tracer_amd import capi
        it.set_rng_mode(capi.VPT_RNG_PIXEL)
    from volume_path_tracer_amd import capi as _capi
    lat_info = None
    if hasattr(_capi.lib(), "vpt_gpu_set_latency_kernel"):  # (A/B runs against older library builds lack it)
        mode, ungated = {"auto": (-1, -1), "off": (0, -1), "on": (1, 1), "gated": (1, 0)}[args.latency_kernel]
        it.set_latency_kernel(mode, ungated)
        lat_info = it.latency_kernel_info()
    if args.compaction is not None:
        it.set_compaction(args.compaction)
    if args.film_order == "atomic":
        it.set_film_order(_capi.VPT_FILM_ATOMIC)
    log(f"[rank {rank}] grids ready in {time.time() - t0:.1f}s: {dens.leaf_count} leaves, "
        f"launch {it.launch_info()}, latency kernel {lat_info}")

    spp = wl.spp
    ranges = D.rank_job_ranges(rank, world, spp, it.jobs_per_wave, args.mode)
    jobs_rank = sum(n for _, n in ranges)
    stream = torch.cuda.current_stream(dev)
    launch_ms = []
    elapsed = max_over_ranks(timed_frames(it, rank, world, spp, args.mode, args.steps, args.warmup, stream, launch_ms),
                             world, sdev)

    kernel_ms = [a.elapsed_time(b) for a, b in launch_ms]
    counters = it.counters()
    samples_rank = counters["samples"]
    assert samples_rank == (wl.cfg.width * wl.cfg.height * jobs_rank // it.jobs_per_wave) * args.steps, samples_rank
    total_samples = sum_over_ranks(samples_rank, world, sdev)
    value = total_samples / elapsed / 1e6
    launches_per_step = max(1, len(ranges))
    film = it.film_host()
    assert (film[..., 3] == D.total_samples_per_pixel(world, spp, args.mode)).all(), "sample-count channel mismatch"
    del it

    strong = None
    if world > 1 and args.strong_configs and args.rng_mode == "reference":
        strong = strong_scaling([c for c in args.strong_configs.split(",") if c], dens, rank, world, dev, sdev,
                                args.steps, args.warmup, stream)

    if rank == 0:
        avg_launch_s = sum(kernel_ms) / len(kernel_ms) / 1e3 / launches_per_step
        bytes_per_launch = algorithmic_bytes(counters) / (args.steps * launches_per_step)
        achieved = bytes_per_launch / avg_launch_s / 1e9
        # PMC-measured HBM bytes of this workload from the newest committed rocprofv3 pass
        # (tools/profile_round.sh): a builder measurement, labelled with its file, not this run's
        pj, traffic_source = newest_profile("*_pmc.json", lambda j: j.get("config") == args.config and j.get("spp") == spp)
        traffic = pj.get("hbm_bytes_per_launch") if pj else None
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        req = request_roofline(args.config, samples_rank / (args.steps * launches_per_step), avg_launch_s, cus)
        pool_mib = (dens.leaf_count + (temp.leaf_count if temp is not None else 0)) * POOL_BYTES_PER_LEAF / 2**20
        req.update(pipe_roofline(args.config, samples_rank / args.steps / launches_per_step / avg_launch_s / cus,
                                 (counters["stencils"] + counters["temp_stencils"]) / samples_rank, pool_mib))
        req.update(mix_roofline(args.config, spp, avg_launch_s, wl.cfg.width * wl.cfg.height * spp,
                                samples_rank / (args.steps * launches_per_step)))
        out = {
            "metric": baseline_metric(),
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.mode,
            "vs_baseline": None,
            "dtype": "f32",
            "data": (f"synthetic ({wl.grid_n}^3 procedural cloud stand-in for "
                     f"{'fire.nvdb + 40*base temperature grid' if wl.temperature else 'wdas_cloud.nvdb'}, SURVEY §8d)"
                     if wl.density_kind == 1 else f"synthetic constant-density {wl.grid_n}^3 grid (SURVEY §8d C2)"),
            "config": {"workload": f"{args.config}: {'fire' if wl.temperature else 'wdas_cloud'}.json "
                                   f"{wl.cfg.width}x{wl.cfg.height}, {spp} spp "
                                   f"{'per GPU' if args.mode == 'weak' else 'per image'}, 8x8 tiles, seed {wl.cfg.seed}",
                       "width": wl.cfg.width, "height": wl.cfg.height, "spp": spp,
                       "jobs_per_step_per_gpu": jobs_rank, "volume": f"synthetic {wl.grid_n}^3 kind {wl.density_kind}",
                       "parallelism": f"wave-sharded x{world} ({args.mode}), RCCL film all-reduce" if world > 1 else "1 GPU",
                       "rng_mode": args.rng_mode, "latency_kernel": args.latency_kernel,
                       "film_order": args.film_order,
                       **({"compaction": args.compaction} if args.compaction is not None else {})},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_source": traffic_source,
                         "kernel": "vpt_integrate_kernel", "avg_launch_ms": round(avg_launch_s * 1e3, 3),
                         "algorithmic_bytes_per_launch": int(bytes_per_launch),
                         "bytes_per_sample": round(algorithmic_bytes(counters) / samples_rank, 2), **req},
            # the production kernel counts the events that price algorithmic bytes
            "counters_per_sample": {k: round(counters[k] / samples_rank, 3)
                                    for k in ("dda_steps", "stencils", "temp_stencils")},
        }
        if strong is not None:
            out["scaling_strong"] = strong
        if dropin is not None:
            if "ms_per_frame" in dropin:
                dropin["vs_one_launch"] = round(out["ms_per_step"] / dropin["ms_per_frame"], 4)
            dfilm = dropin.pop("_film", None)
            if dfilm is not None and world == 1 and args.mode == "weak" and dfilm.shape == film.shape:
                # the drop-in's last frame against this process's one-launch frame (both the reference's film, bit
                # for bit, when both are in wave order)
                import numpy as np
                differ = int((dfilm.view(np.uint32) != film.view(np.uint32)).any(axis=-1).sum())
                dropin["bit_identical_to_one_launch"] = differ == 0
                dropin["pixels_differing_from_one_launch"] = differ
            out["dropin"] = dropin
        if world == 1 and not args.no_cpu_baseline:
            cb, ref_film, k = cpu_baseline(wl, dens, temp, args.cpu_budget)
            out["cpu_baseline"] = cb
            out["parity"] = film_parity(wl, dens, temp, ref_film, k, dev.index)
            out["speedup_vs_cpu_baseline"] = round(value / cb["value"], 1) if cb["value"] else None
            ne = cb["node_extrapolated"]["value"]
            out["speedup_vs_cpu_node_extrapolated"] = round(value / ne, 1) if ne else None
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
