"""tools/ubench/gather output (+ its rocprofv3 --pmc TCP_TCC_READ_REQ_sum pass) -> profiles/<tag>_gather_ceiling.json.

The ceiling the bench's roofline.request_frac divides by: the highest L1->L2 read-request rate per CU
that divergent 4-byte per-lane gathers reach from an L2-resident table (the walk-word pattern), over
chains per lane and waves per SIMD.  Lane loads convert to requests with the PMC pass of the same
binary (requests per lane load, ~1: every random 4-B load of a 1.2 MiB table misses the 32 KB L1).
Usage: python tools/gather_ceiling.py <tag> <gather.txt> [<pmc dir>]"""
import csv
import json
import sys
from pathlib import Path

tag, txt = sys.argv[1], Path(sys.argv[2])
pmc = Path(sys.argv[3]) if len(sys.argv) > 3 else None
rows, active = [], []
for line in txt.read_text().splitlines():
    p = line.split()
    if len(p) == 4 and p[0][0].isdigit():
        rows.append({"table_mib": float(p[0]), "chains": int(p[1]), "waves": int(p[2]), "gload_per_s_per_cu": float(p[3])})
    elif len(p) == 6 and p[0][0].isdigit():
        active.append({"table_mib": float(p[0]), "chains": int(p[1]), "waves": int(p[2]), "active_lanes": int(p[3]),
                       "gload_per_s_per_cu": float(p[4]), "ginst_per_s_per_cu": float(p[5])})
l2 = [r for r in rows if r["table_mib"] < 4]
best = max(l2, key=lambda r: r["gload_per_s_per_cu"])
req_per_load = None
if pmc is not None:  # the `gather calib` run: 2 dispatches of one config, lane loads each in its log
    per = {}
    for f in pmc.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "chase" in r["Kernel_Name"]:
                per.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    loads = None
    for f in list(pmc.parent.glob("*.log")) + list(pmc.glob("*.log")):
        for line in f.read_text().splitlines():
            if line.startswith("calib lane_loads_per_launch"):
                loads = float(line.split()[2])
    if loads and per.get("TCP_TCC_READ_REQ_sum"):
        req = per["TCP_TCC_READ_REQ_sum"]
        acc = per.get("TCP_TOTAL_CACHE_ACCESSES_sum", [0.0])
        req_per_load = {"lane_loads_per_launch": loads, "requests_per_launch": sum(req) / len(req),
                        "requests_per_lane_load": sum(req) / len(req) / loads,
                        "l1_accesses_per_lane_load": sum(acc) / len(acc) / loads}
rpl = req_per_load["requests_per_lane_load"] if req_per_load else 1.0
out = {"tool": "tools/ubench/gather.hip", "cus": 256,
       "ceiling_lane_loads_per_s_per_cu": best["gload_per_s_per_cu"] * 1e9, "ceiling_at": best,
       "ceiling_l1_to_l2_requests_per_s_per_cu": best["gload_per_s_per_cu"] * 1e9 * rpl,
       "pmc_calibration": req_per_load, "rows": rows, "partly_active_wavefronts": active}
Path("profiles").mkdir(exist_ok=True)
Path(f"profiles/{tag}_gather_ceiling.json").write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps({k: out[k] for k in ("ceiling_lane_loads_per_s_per_cu", "ceiling_l1_to_l2_requests_per_s_per_cu",
                                     "ceiling_at", "pmc_calibration")}, indent=1))
