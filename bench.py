#!/usr/bin/env python3
"""Benchmark: Msamples/s of the volumetric path-tracing integrator on BASELINE.json's headline
workload (configs[2]: wdas_cloud.json at 1920x1080, 256 spp, one MI355X), on the synthetic 512^3
cloud stand-in (the reference's wdas_cloud.nvdb is not available).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]

One step = one full frame (every wave of the configuration) rendered into a zeroed film on every
rank, plus — for N > 1 — the RCCL sum of the films over xGMI.  Multi-GPU is weak scaling: rank r
renders waves r*spp+1 .. (r+1)*spp of the same job space (independent RNG streams per job id), so
the per-GPU work is fixed and the reduced film is an N*spp-sample image.

The JSON line also carries:
  roofline      the integrator kernel's algorithmic bytes per launch (SURVEY §8d:
                32*stencils + 8*dda_steps + 32*temp_stencils + 32*samples, from the kernel's own
                event counters) / its average launch time (HIP events on the launch stream), against
                the 8 TB/s HBM peak; `traffic` = PMC-measured HBM bytes per launch from
                profiles/<round>_pmc.json when that file exists (rocprofv3 --pmc pass), else null.
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


def cpu_baseline(wl, dens, temp, budget_s: float = 12.0):
    """Oracle worker pool on this host: whole waves of the workload's frame until ~budget_s."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O

    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    threads = max(1, min(16, aff, os.cpu_count() or 1))
    od = O.OracleGrid(dens, fix_majorants=True)
    ot = O.OracleGrid(temp, fix_majorants=False) if temp is not None else None
    cfg = wl.cfg.copy()
    waves, total_ms = 0, 0.0
    samples = cfg.width * cfg.height
    while waves < 16:
        film, ms, _ = O.render_pool(cfg, od, ot, 1, threads)
        waves += 1
        total_ms += ms
        if total_ms / 1e3 >= budget_s:
            break
        # each call renders wave 1 again (same jobs): a fixed, repeatable sample of the frame
        if total_ms / waves * (waves + 1) / 1e3 > 2.5 * budget_s:
            break
    rate = waves * samples / (total_ms / 1e3) / 1e6
    return {"value": round(rate, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{waves} x wave 1 of {cfg.width}x{cfg.height} ({waves * samples} samples), "
                      f"oracle worker pool, {threads} threads, {total_ms / 1e3:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--spp", type=int, default=None, help="override waves per step (default: the config's)")
    ap.add_argument("--mode", choices=["weak", "strong"], default="weak",
                    help="weak: each rank renders its own spp waves; strong: the spp waves are dealt across ranks")
    ap.add_argument("--rng-mode", choices=["reference", "pixel"], default="reference",
                    help="pixel = throughput mode (per-pixel streams; not the reference's samples)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    from volume_path_tracer_amd import distributed as D
    from volume_path_tracer_amd.render import Integrator
    from volume_path_tracer_amd.scenes import SynthGrid, workload

    wl = workload(args.config, spp=args.spp)
    t0 = time.time()
    dg = SynthGrid(wl.density_kind, wl.grid_n)
    tg = SynthGrid(2, wl.grid_n) if wl.temperature else None
    dens, temp = dg.grid(copy=False), (tg.grid(copy=False) if tg else None)
    it = Integrator(wl.cfg, dens, temp, device=dev.index)
    if args.rng_mode == "pixel":
        from volume_path_tracer_amd import capi
        it.set_rng_mode(capi.VPT_RNG_PIXEL)
    log(f"[rank {rank}] grids ready in {time.time() - t0:.1f}s: {dens.leaf_count} leaves, "
        f"launch {it.launch_info()}")

    spp = wl.spp
    ranges = D.rank_job_ranges(rank, world, spp, it.jobs_per_wave, args.mode)
    jobs_rank = sum(n for _, n in ranges)
    stream = torch.cuda.current_stream(dev)
    launch_ms = []

    def step(timed: bool):
        it.film.zero_()
        for b, n in ranges:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev0.record(stream)
            it.render_jobs(b, n, stream=stream)
            ev1.record(stream)
            if timed:
                launch_ms.append((ev0, ev1))
        D.reduce_film(it.film)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    it.counters(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    kernel_ms = [a.elapsed_time(b) for a, b in launch_ms]
    counters = it.counters()
    area = int(wl.cfg.tile_size[0] * wl.cfg.tile_size[1])
    samples_rank = counters["samples"]
    assert samples_rank == (wl.cfg.width * wl.cfg.height * jobs_rank // it.jobs_per_wave) * args.steps, samples_rank
    t = torch.tensor([samples_rank], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    total_samples = int(t.item())
    value = total_samples / elapsed / 1e6
    launches_per_step = len(ranges)

    if rank == 0:
        avg_launch_s = sum(kernel_ms) / len(kernel_ms) / 1e3
        bytes_per_launch = algorithmic_bytes(counters) / (args.steps * launches_per_step)
        achieved = bytes_per_launch / avg_launch_s / 1e9
        traffic = None
        pmc = sorted((ROOT / "profiles").glob("*_pmc.json"))
        if pmc:
            try:
                pj = json.loads(pmc[-1].read_text())
                if pj.get("config") == args.config and pj.get("spp") == spp:
                    traffic = pj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        film = it.film_host()
        assert (film[..., 3] == D.total_samples_per_pixel(world, spp, args.mode)).all(), "sample-count channel mismatch"
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
                       "rng_mode": args.rng_mode},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "kernel": "vpt_integrate_kernel", "avg_launch_ms": round(avg_launch_s * 1e3, 3),
                         "algorithmic_bytes_per_launch": int(bytes_per_launch),
                         "bytes_per_sample": round(algorithmic_bytes(counters) / samples_rank, 2)},
            # the production kernel counts the events that price algorithmic bytes
            "counters_per_sample": {k: round(counters[k] / samples_rank, 3)
                                    for k in ("dda_steps", "stencils", "temp_stencils")},
        }
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(wl, dens, temp, args.cpu_budget)
            out["cpu_baseline"] = cb
            out["speedup_vs_cpu_baseline"] = round(value / cb["value"], 1) if cb["value"] else None
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
