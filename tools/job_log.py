"""Per-job timing of one frame with the diagnostic VPT_JOB_LOG build (tile, fetch time, end time,
hardware slot per job; s_memrealtime, 100 MHz): drain profile of the launch and measured per-tile costs.
    VPT_LIB=.../libvpt_amd_joblog.so python tools/job_log.py [--config c3] [--out gpurun_out/joblog]"""
import argparse, json, sys
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--spp", type=int, default=None)
ap.add_argument("--out", default="gpurun_out/joblog")
ap.add_argument("--alone", type=int, default=0,
                help="then render the N longest jobs again one at a time (one lane on the device), on the "
                     "throughput and the latency kernel: their duration without the full launch's contention")
a = ap.parse_args()
import torch
from volume_path_tracer_amd.render import Integrator
from volume_path_tracer_amd.scenes import SynthGrid, workload
wl = workload(a.config, spp=a.spp)
dg = SynthGrid(wl.density_kind, wl.grid_n); tg = SynthGrid(2, wl.grid_n) if wl.temperature else None
it = Integrator(wl.cfg, dg.grid(copy=False), tg.grid(copy=False) if tg else None)
T = it.jobs_per_wave; jobs = T * wl.spp
import ctypes as C
from volume_path_tracer_amd import capi
log = torch.zeros(jobs * 4, dtype=torch.float32, device="cuda")
def frame():  # the job log travels in the records argument of the VPT_JOB_LOG build (16 B per job)
    capi.check(capi.lib().vpt_gpu_render_jobs_records(it.h, 0, jobs, C.c_void_p(it.film.data_ptr()),
                                                      C.c_void_p(log.data_ptr()), C.c_void_p(None)), "render")
    torch.cuda.synchronize()
frame()   # warm-up (same order)
log.zero_(); it.film.zero_()
frame()
L = log.view(torch.int32).cpu().numpy().view(np.uint32).reshape(jobs, 4).astype(np.int64)
tile, t0, t1, hw = L[:, 0], L[:, 1], L[:, 2], L[:, 3]
# s_memrealtime is read per XCD; blocks are dealt round-robin to the 8 XCDs: time each XCD from its
# own first fetch (every XCD starts its resident blocks at launch)
xcd = (hw >> 8) % 8
xcd_span = {}
for x in range(8):
    m = xcd == x
    b = t0[m].min()
    t0[m] -= b; t1[m] -= b
    xcd_span[x] = float(t1[m].max() / 1e5)
span = t1.max()
dur = t1 - t0
lanes = it.launch_info()[0] * it.launch_info()[1]
# running jobs over time (0.5 ms bins = 50000 ticks of the 100 MHz clock)
B = 50000
nb = int(span // B) + 1
run = np.zeros(nb + 1)
np.add.at(run, t0 // B, 1); np.add.at(run, t1 // B, -1)
run = np.cumsum(run)[:nb]
first_idle = int(np.argmax(run < 0.95 * lanes)) * 0.5   # ms: running jobs fall below 95 % of the lanes
busy = float(dur.sum() / (lanes * span))                  # lane-time with a job / lane-time of the launch
cost = np.zeros(T); np.add.at(cost, tile, dur.astype(np.float64))
est, _ = it.tile_costs()
rc = np.corrcoef(np.argsort(np.argsort(cost)), np.argsort(np.argsort(est)))[0, 1]
last = np.argsort(t1)[-2000:]
blk = hw >> 8
first = np.full(blk.max() + 1, np.iinfo(np.int64).max); np.minimum.at(first, blk, t0)
lastend = np.zeros(blk.max() + 1, np.int64); np.maximum.at(lastend, blk, t1)
out = {"block_first_fetch_ms_pct": {p: float(np.percentile(first, p) / 1e5) for p in (0, 10, 50, 90, 100)},
       "block_last_end_ms_pct": {p: float(np.percentile(lastend, p) / 1e5) for p in (0, 10, 50, 90, 100)},
       "first_fetch_vs_block_corr": float(np.corrcoef(np.arange(len(first)), first)[0, 1]),
       "xcd_span_ms": xcd_span, "config": a.config, "jobs": int(jobs), "lanes": int(lanes), "span_ms": span / 1e5,
       "first_below_95pct_lanes_ms": first_idle, "lane_busy_fraction": busy, "drain_ms": span / 1e5 - first_idle,
       "job_ms_mean": float(dur.mean() / 1e5), "job_ms_p99": float(np.percentile(dur, 99) / 1e5),
       "job_ms_max": float(dur.max() / 1e5),
       # the launch's lower bounds: the longest single job (one lane traces it serially) and the work spread
       # evenly over every lane; span / max(both) is how far the drain is from ideal
       "work_over_lanes_ms": float(dur.sum() / lanes / 1e5),
       "ideal_span_ms": float(max(dur.max(), dur.sum() / lanes) / 1e5),
       "span_over_ideal": float(span / max(dur.max(), dur.sum() / lanes)),
       "last_2000_jobs_start_ms_min": float(t0[last].min() / 1e5), "last_2000_jobs_dur_ms_max": float(dur[last].max() / 1e5),
       "rank_corr_measured_vs_estimated_cost": float(rc),
       "running_jobs_at_ms": {f"{x:.0f}": float(run[int(x * 2)]) for x in np.linspace(0, span / 1e5 - 0.5, 41)}}
if a.alone:
    # the longest jobs alone: a launch of one job (its lane has a SIMD to itself); each twice, the second kept
    one = torch.zeros(4, dtype=torch.float32, device="cuda")
    def alone_ms(jid):
        for _ in range(2):
            one.zero_()
            capi.check(capi.lib().vpt_gpu_render_jobs_records(it.h, int(jid), 1, C.c_void_p(it.film.data_ptr()),
                                                              C.c_void_p(one.data_ptr()), C.c_void_p(None)), "render")
            torch.cuda.synchronize()
        r = one.view(torch.int32).cpu().numpy().view(np.uint32).astype(np.int64)
        assert r[0] == tile[jid], ("the one-job launch rendered another tile", int(r[0]), int(tile[jid]))
        return float((r[2] - r[1]) / 1e5)
    top = np.argsort(dur)[::-1][:a.alone]
    rows = []
    for lat in (0, 1):
        it.set_latency_kernel(lat, 0)
        rows.append([alone_ms(j) for j in top])
    it.set_latency_kernel(-1, 0)
    out["longest_jobs"] = [{"jid": int(j), "tile": int(tile[j]), "in_launch_ms": float(dur[j] / 1e5),
                            "start_ms": float(t0[j] / 1e5), "alone_ms": rows[0][i], "alone_latency_kernel_ms": rows[1][i]}
                           for i, j in enumerate(top)]
Path(a.out).mkdir(parents=True, exist_ok=True)
np.save(Path(a.out) / f"tile_cost_{a.config}.npy", cost.astype(np.float32))
Path(a.out, f"summary_{a.config}.json").write_text(json.dumps(out, indent=1))
print(json.dumps(out))
