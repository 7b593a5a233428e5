"""All event counters per sample for a workload (debug/records launch; timing irrelevant).
    python tools/counters.py --config c3 --spp 2"""
import argparse, json, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--spp", type=int, default=2)
a = ap.parse_args()
import torch
from volume_path_tracer_amd.render import Integrator
from volume_path_tracer_amd.scenes import SynthGrid, workload
wl = workload(a.config, spp=a.spp)
dg = SynthGrid(wl.density_kind, wl.grid_n); tg = SynthGrid(2, wl.grid_n) if wl.temperature else None
it = Integrator(wl.cfg, dg.grid(copy=False), tg.grid(copy=False) if tg else None)
T = wl.cfg.jobs_per_wave()
jobs = T * a.spp
rec = torch.empty((jobs * wl.cfg.tile_size[0] * wl.cfg.tile_size[1], 3), device="cuda:0")
it.counters(reset=True)
it.render_jobs(0, jobs, records=rec)
torch.cuda.synchronize()
c = it.counters(reset=True)
n = c["samples"]
print(json.dumps({"config": a.config, "spp": a.spp, "samples": n,
                  "per_sample": {k: round(v / n, 4) for k, v in c.items()}}))
