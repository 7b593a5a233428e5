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
g = summary.get
fetch_kb, write_kb = g("FETCH_SIZE"), g("WRITE_SIZE")
# Fabric read bytes from the size-resolved request counters (no width assumption): every L2 miss
# leaves the XCD as one 32-, 64- or 128-byte request.  Infinity-Cache hits are included (the counters
# sit on the L2's memory side).  Writes: WRITE_SIZE, exact for fp32 atomics (MI355X_MICROARCH.md).
read_bytes = None
if g("TCC_EA0_RDREQ_32B_sum") is not None:
    read_bytes = 32 * g("TCC_EA0_RDREQ_32B_sum", 0) + 64 * g("TCC_EA0_RDREQ_64B_sum", 0) + 128 * g("TCC_EA0_RDREQ_128B_sum", 0)
traffic = None
if read_bytes is not None and write_kb is not None:
    traffic = int(read_bytes + write_kb * 1024)
elif fetch_kb is not None and write_kb is not None:
    traffic = int((2 * fetch_kb + write_kb) * 1024)
out = {"config": config, "spp": spp, "kernel": "vpt_integrate_kernel", "launches_averaged": len(vals.get("FETCH_SIZE", [])),
       "counters_per_launch": {k: round(v, 1) for k, v in summary.items()},
       "fabric_read_bytes_per_launch": None if read_bytes is None else int(read_bytes),
       "fetch_size_x2_bytes_per_launch": None if fetch_kb is None else int(2 * fetch_kb * 1024),
       "hbm_bytes_per_launch": traffic,
       "method": "rocprofv3 --pmc, one pass per counter group, one C3 launch; traffic = 32*RDREQ_32B + 64*RDREQ_64B "
                 "+ 128*RDREQ_128B (TCC_EA0, size-resolved fabric read requests) + WRITE_SIZE*1024; "
                 "Infinity-Cache hits are counted (they sit behind the same requests)"}
Path("profiles").mkdir(exist_ok=True)
Path(f"profiles/{tag}_pmc.json").write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out))
