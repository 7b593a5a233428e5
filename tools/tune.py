"""GPU tuning sweeps (timing only): frames of a config at reduced spp under scheduling knobs / library
builds (VPT_LIB).  Results never depend on the knobs (every job keeps its jid and RNG stream).

    python tools/tune.py --spp 8 --gates 1:1,16:16 [--blocks 256,1792] [--lat 0:1:65:1:1,...]
    python tools/tune.py --preset latency            # a named sweep (PRESETS below), JSON rows to stdout

--gates gate_min:gate_idle[:gate_eval[:gate_walk]] (vpt_gpu_set_tuning); --lat
wave_lanes:gate_min:gate_idle:gate_eval:gate_walk (vpt_gpu_set_latency_tuning); --blocks grid sizes
(0 = resident capacity).  --profile prints the -DVPT_PROFILE build's SIMT / wave-time profile."""
import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

# Named sweeps (the r02 one-off scripts, folded in): each entry is one tune.py argument list.
_C1_LAT = "64:6:8:36:4,0:6:8:36:4,0:1:65:1:1,0:1:65:1:0,0:1:65:8:2,0:2:16:8:2"
PRESETS = {
    # latency-bound launches: C1 (4 096 jobs) over grid sizes and latency knobs, C2's partly filled launch
    "latency": [["--config", "c1", "--spp", "4", "--gates", "6:8:36:4", "--blocks", "256,512,1024,1792", "--lat", _C1_LAT, "--reps", "3"],
                ["--config", "c2", "--spp", "64", "--gates", "6:8:36:4", "--blocks", "768,1792",
                 "--lat", "0:6:8:36:4,0:1:65:1:1,0:2:16:8:2", "--reps", "2"]],
    # where spreading a launch over the full grid stops paying: C1 frames of 4..64 spp, spread vs 256 blocks
    "latency-threshold": [a for s in (4, 8, 16, 32, 48, 64) for a in (
        ["--config", "c1", "--spp", str(s), "--gates", "6:8:36:4", "--blocks", "1792", "--reps", "3"],
        ["--config", "c1", "--spp", str(s), "--gates", "6:8:36:4", "--blocks", "256", "--lat", "64:6:8:36:4", "--reps", "3"])],
    # job lanes per wavefront in latency launches (wave_lanes 1 / 2 / 3 / auto)
    "c1-lanes": [["--config", "c1", "--spp", "4", "--gates", "6:8:36:4", "--blocks", "1024,1280,1536,1792", "--lat", "1:1:65:1:1,2:1:65:1:1", "--reps", "3"],
                 ["--config", "c1", "--spp", "8", "--gates", "6:8:36:4", "--blocks", "1792", "--lat", "1:1:65:1:1,2:1:65:1:1,3:1:65:1:1", "--reps", "3"]]
    + [["--config", "c1", "--spp", str(s), "--gates", "6:8:36:4", "--blocks", "1792",
        "--lat", "1:1:65:1:1,2:1:65:1:1,3:1:65:1:1,0:1:65:1:1", "--reps", "2"] for s in (16, 32, 48)],
    # grid sizes of C2's partly filled launch (262 144 jobs) and C1's latency gates
    "small-launch": [["--config", "c2", "--spp", "64", "--gates", "6:8:36:4", "--blocks", "512,640,768,1024,1280", "--reps", "2"],
                     ["--config", "c1", "--spp", "4", "--gates", "6:8:36:4", "--blocks", "1792",
                      "--lat", "0:1:65:1:1,0:1:65:2:1,0:1:65:1:2,0:1:65:4:1,0:1:65:1:4,0:2:65:1:1", "--reps", "3"]],
    # C2 on the latency kernel with the context's gates (r04): gates and blocks per CU
    "c2-lat": [["--config", "c2", "--spp", "64", "--lat-kernel", "1", "--lat-ungated", "0", "--blocks", "512,768,1024",
                "--gates", "6:8:36:4,4:8:36:4,8:8:36:4,6:4:36:4,6:16:36:4,6:8:24:4,6:8:48:4,6:8:36:2,6:8:36:8", "--reps", "3"],
               ["--config", "c2", "--spp", "64", "--lat-kernel", "0", "--blocks", "512", "--gates", "6:8:36:4", "--reps", "3"]],
    # the full-occupancy gates of the C3 / C4 frames
    "gates": [["--config", c, "--spp", "32", "--gates", "6:8:36:4,4:8:36:4,8:8:36:4,6:12:36:4,6:8:32:4,6:8:40:4,6:8:36:2,6:8:36:8",
               "--reps", "2"] for c in ("c3", "c4")],
}


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", choices=sorted(PRESETS), default=None)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--gates", default="16:16")
    ap.add_argument("--blocks", default="0")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--lat", default="", help="latency-launch knobs wave_lanes:gate_min:gate_idle:gate_eval:gate_walk, comma-separated")
    ap.add_argument("--lat-kernel", type=int, default=-1, help="vpt_gpu_set_latency_kernel mode (-1 auto, 0 off, 1 on)")
    ap.add_argument("--lat-ungated", type=int, default=-1, help="its ungated flag (-1 keep)")
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--compact", default="0", help="live-path compaction periods to sweep (comma-separated; 0 = off)")
    ap.add_argument("--rng-mode", default="reference")
    ap.add_argument("--order", type=int, default=-1, help="job order mode (-1: library default)")
    ap.add_argument("--tail", type=int, default=0, help="VPT_ORDER_COST_TAIL tile-major waves (0: auto)")
    ap.add_argument("--tile-costs", default=None, help=".npy of per-tile costs for the job order (vpt_gpu_set_tile_costs)")
    ap.add_argument("--perm", default="", help="explicit job order: 'same-tile' = each tile's jobs of all waves consecutively, "
                    "costliest tile first (the lanes of a wavefront trace one tile's pixels at different spp)")
    return ap


def sweep(a):
    import torch

    from volume_path_tracer_amd.render import Integrator
    from volume_path_tracer_amd.scenes import SynthGrid, workload

    wl = workload(a.config, spp=a.spp)
    dg = SynthGrid(wl.density_kind, wl.grid_n)
    tg = SynthGrid(2, wl.grid_n) if wl.temperature else None
    it = Integrator(wl.cfg, dg.grid(copy=False), tg.grid(copy=False) if tg else None)
    base_blocks = it.launch_info()[0]
    it.set_latency_kernel(a.lat_kernel, a.lat_ungated)
    if a.rng_mode == "pixel":
        from volume_path_tracer_amd import capi
        it.set_rng_mode(capi.VPT_RNG_PIXEL)
    if a.order >= 0:
        it.set_job_order(a.order)
    it.set_job_order_tail(a.tail)
    if a.tile_costs:
        import numpy as np
        it.set_tile_costs(np.load(a.tile_costs))
    if a.perm == "same-tile":
        import numpy as np
        T = wl.cfg.jobs_per_wave()
        tiles = np.argsort(-it.tile_costs()[0], kind="stable").astype(np.int64)
        it.set_job_permutation((np.arange(a.spp, dtype=np.int64)[None, :] * T + tiles[:, None]).reshape(-1))
    it.render_waves(1, 1)
    torch.cuda.synchronize()
    if a.profile:
        it.profile(reset=True)
    for g in a.gates.split(","):
        parts = list(map(int, g.split(":")))
        gm, gi = parts[0], parts[1]
        ge = parts[2] if len(parts) > 2 else 1
        gw = parts[3] if len(parts) > 3 else 0
        for b, lat, cmp in [(b, l, c) for b in map(int, a.blocks.split(",")) for l in (a.lat.split(",") if a.lat else [""])
                            for c in map(int, a.compact.split(","))]:
            it.set_tuning(gm, gi, b if b > 0 else base_blocks, ge, gw)
            it.set_compaction(cmp)
            if lat:
                it.set_latency_tuning(*map(int, lat.split(":")))
            best = 1e9
            for _ in range(a.reps):
                it.film.zero_()
                torch.cuda.synchronize()
                t = time.perf_counter()
                it.render_waves(1, a.spp)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t)
            if a.profile:
                print(json.dumps({"gate": g, "profile": it.profile(reset=True)}), flush=True)
            print(json.dumps({"lib": os.environ.get("VPT_LIB", "default"), "config": a.config, "order": a.order, "tail": a.tail, "perm": a.perm,
                              "gate": g, "lat": lat, "lat_kernel": [a.lat_kernel, a.lat_ungated], "compact": cmp,
                              "exchanged": it.counters(reset=True).get("exchanged", 0),
                              "blocks": b or base_blocks, "spp": a.spp, "ms": round(best * 1e3, 2),
                              "Msps": round(wl.cfg.width * wl.cfg.height * a.spp / best / 1e6, 2)}), flush=True)
    del it


def main():
    a = parser().parse_args()
    if a.preset:
        for argv in PRESETS[a.preset]:
            sweep(parser().parse_args(argv))
    else:
        sweep(a)


if __name__ == "__main__":
    main()
