"""Job-order experiments on the full C3 frame through vpt_gpu_set_job_permutation (samples never depend
on the order, only the launch's drain does).  Costs: measured per-tile job times (tools/job_log.py) or
the built-in estimates.
    python tools/order_lab.py [--costs gpurun_out/joblog/tile_cost_c3.npy] [--reps 2]"""
import argparse, json, sys, time
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--costs", default=None)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--only", default=None)
ap.add_argument("--regions", default=None, help="region-major orders with these region sizes (tiles), e.g. 1024,4096")
ap.add_argument("--blocks", default=None, help="cost-tail orders over b x b blocks of adjacent tiles, e.g. 4,8")
ap.add_argument("--tails", default=None, help="with --regions: region-major curve orders ending in the cost tail of these wave counts")
a = ap.parse_args()
import torch
from volume_path_tracer_amd.render import Integrator
from volume_path_tracer_amd.scenes import SynthGrid, workload
wl = workload(a.config)
dg = SynthGrid(wl.density_kind, wl.grid_n); tg = SynthGrid(2, wl.grid_n) if wl.temperature else None
it = Integrator(wl.cfg, dg.grid(copy=False), tg.grid(copy=False) if tg else None)
T, W = it.jobs_per_wave, wl.spp
lanes = it.launch_info()[0] * it.launch_info()[1]
est, _ = it.tile_costs()
cost = np.load(a.costs).astype(np.float64) if a.costs else est.astype(np.float64)
rank = np.argsort(-cost, kind="stable").astype(np.int64)


def cost_tail(rank, n_waves, tail, waves0=0):
    """vpt_integrator.h ordered_job: wave-major costliest-first, then `tail` waves tile-major in groups of 64."""
    head = (np.arange(waves0, n_waves - tail)[:, None] * T + rank[None, :]).ravel()
    full = len(rank) // 64
    g = rank[: full * 64].reshape(full, 64)
    tw = np.arange(n_waves - tail, n_waves)
    body = (tw[None, :, None] * T + g[:, None, :]).reshape(-1)
    rest = (tw[:, None] * T + rank[full * 64:][None, :]).ravel()
    return np.concatenate([head, body, rest])


auto_tail = min(W, (6 * lanes + T - 1) // T)
orders = {"builtin": None, "perm_current": cost_tail(rank, W, auto_tail)}
for K in (128, 512, 2048):
    top = rank[:K]
    topset = np.zeros(T, bool); topset[top] = True
    tw = np.arange(W - auto_tail, W)
    front = (tw[None, :, None] * T + top.reshape(-1, 64)[:, None, :]).reshape(-1) if K % 64 == 0 else None
    base = cost_tail(rank, W, auto_tail)
    keep = ~np.isin(base, front)
    orders[f"front_top{K}_tail"] = np.concatenate([front, base[keep]])
for tl in (auto_tail // 2, auto_tail * 2):
    orders[f"tail{tl}"] = cost_tail(rank, W, min(W, tl))


def morton(tx, ty):
    """Interleaved bits of (tx, ty): a Z-order curve over the tile grid."""
    code = np.zeros_like(tx, dtype=np.int64)
    for b in range(12):
        code |= ((tx >> b) & 1) << (2 * b) | ((ty >> b) & 1) << (2 * b + 1)
    return code


def region_major(G, group_order="cost"):
    """Regions of G tiles compact in the image (consecutive along a Z-order curve): every wave of a region
    before the next region, so the lanes in flight trace one region's frustum through the volume and the
    stencil pool lines they touch are reused from L2 / MALL; within a region and wave the tiles costliest
    first (64 consecutive items = 64 different tiles: no film-atomic conflicts).  Regions costliest first
    (group_order "cost") so the launch drains on cheap regions, or along the curve ("curve")."""
    ntx = int(np.ceil(wl.cfg.width / wl.cfg.tile_size[0]))
    tiles = np.arange(T)
    z = np.argsort(morton(tiles % ntx, tiles // ntx), kind="stable")
    groups = [z[i:i + G] for i in range(0, T, G)]
    if group_order == "cost":
        groups.sort(key=lambda g: -cost[g].sum() / len(g))
    parts = []
    for g in groups:
        g = g[np.argsort(-cost[g], kind="stable")]
        parts.append((np.arange(W)[:, None] * T + g[None, :]).ravel())
    return np.concatenate(parts)


def region_then_tail(G, tail):
    """region_major along the curve for the first W - tail waves, then the built-in cost tail (the last `tail`
    waves over all tiles, costliest first in groups of 64) so the launch drains on cheap jobs."""
    ntx = int(np.ceil(wl.cfg.width / wl.cfg.tile_size[0]))
    tiles = np.arange(T)
    z = np.argsort(morton(tiles % ntx, tiles // ntx), kind="stable")
    parts = []
    for i in range(0, T, G):
        g = z[i:i + G]
        g = g[np.argsort(-cost[g], kind="stable")]
        parts.append((np.arange(W - tail)[:, None] * T + g[None, :]).ravel())
    tl = cost_tail(rank, W, tail, waves0=W - tail)
    return np.concatenate(parts + [tl])


def block_rank(b):
    """Tiles grouped into b x b blocks of adjacent tiles (64 = one wavefront's fetch for b = 8), blocks by
    descending mean estimated cost, tiles raster order within a block: a rank list for cost_tail whose
    consecutive items are neighbouring tiles, so the lanes that fetch together trace nearby primary rays."""
    ntx = int(np.ceil(wl.cfg.width / wl.cfg.tile_size[0]))
    tiles = np.arange(T)
    bx, by = (tiles % ntx) // b, (tiles // ntx) // b
    key = by * (ntx // b + 1) + bx
    order = np.argsort(key, kind="stable")
    blocks = np.split(order, np.flatnonzero(np.diff(key[order])) + 1)
    blocks.sort(key=lambda g: -cost[g].mean())
    return np.concatenate(blocks).astype(np.int64)


if a.blocks:
    orders = {"builtin": None}
    for b in map(int, a.blocks.split(",")):
        orders[f"blocks{b}_cost_tail"] = cost_tail(block_rank(b), W, auto_tail)
    orders["builtin_again"] = None
if a.regions:
    orders = {"builtin": None}
    for G in map(int, a.regions.split(",")):
        if a.tails:
            for t in map(int, a.tails.split(",")):
                orders[f"region{G}_curve_tail{t}"] = region_then_tail(G, t)
        else:
            orders[f"region{G}_cost"] = region_major(G, "cost")
            orders[f"region{G}_curve"] = region_major(G, "curve")
    orders["builtin_again"] = None
res = {}
for name, perm in orders.items():
    if a.only and name not in a.only.split(","):
        continue
    if perm is not None:
        assert perm.size == T * W and np.unique(perm).size == perm.size
    it.set_job_permutation(perm)
    it.film.zero_(); it.render_waves(1, W); torch.cuda.synchronize()
    best = 1e9
    for _ in range(a.reps):
        it.film.zero_(); torch.cuda.synchronize(); t = time.perf_counter()
        it.render_waves(1, W); torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    assert (it.film_host()[..., 3] == W).all()
    res[name] = round(best * 1e3, 2)
    print(json.dumps({"order": name, "ms": res[name], "costs": a.costs or "estimated"}), flush=True)
