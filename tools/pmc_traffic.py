"""Summarise rocprofv3 --pmc passes of `bench.py --steps 1 --warmup 0` into profiles/<tag>_pmc.json.

HBM bytes per integrator launch, corrected as MI355X_MICROARCH.md §HBM prescribes for gfx950:
FETCH_SIZE counts 128-B read requests at 64 B (x2 before comparing with bytes); WRITE_SIZE is
exact for fp32 atomics / 16-B stores.  traffic = (2*FETCH_SIZE + WRITE_SIZE) * 1024.
Usage: python tools/pmc_traffic.py <tag> <config> <spp> <pass_dir>...
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

tag, config, spp, dirs = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4:]
vals = defaultdict(list)
for d in dirs:
    for f in Path(d).rglob("*counter_collection.csv"):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if "integrate" in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (disp, name), v in per.items():
            vals[name].append(v)
summary = {k: (sum(v) / len(v)) for k, v in vals.items()}
fetch_kb, write_kb = summary.get("FETCH_SIZE"), summary.get("WRITE_SIZE")
traffic = None
if fetch_kb is not None and write_kb is not None:
    traffic = int((2 * fetch_kb + write_kb) * 1024)
out = {"config": config, "spp": spp, "kernel": "vpt_integrate_kernel", "launches_averaged": len(vals.get("FETCH_SIZE", [])),
       "counters_per_launch": {k: round(v, 1) for k, v in summary.items()},
       "hbm_bytes_per_launch": traffic,
       "method": "rocprofv3 --pmc, one pass per counter group; traffic = (2*FETCH_SIZE + WRITE_SIZE)*1024 "
                 "(gfx950 FETCH_SIZE tallies 128-B requests at 64 B; Infinity-Cache hits are counted)"}
Path("profiles").mkdir(exist_ok=True)
Path(f"profiles/{tag}_pmc.json").write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out))
