"""Summarise tools/sq_counters.sh output: python tools/sq_summary.py <outdir> [samples]"""
import csv, sys, collections
from pathlib import Path
d = Path(sys.argv[1]); samples = float(sys.argv[2]) if len(sys.argv) > 2 else 1920 * 1080 * 256
agg = collections.defaultdict(float)
for f in d.rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "integrate" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(agg):
    print(f"{k:28s} {agg[k]:18.4g}   per sample {agg[k] / samples:10.2f}")
if agg.get("SQ_WAVE_CYCLES"):
    print("VALU active / wave cycles", round(agg["SQ_ACTIVE_INST_VALU"] / agg["SQ_WAVE_CYCLES"], 3))
    print("wait_any / wave cycles", round(agg["SQ_WAIT_ANY"] / agg["SQ_WAVE_CYCLES"], 3))
    print("VALU lane utilisation", round(agg.get("SQ_THREAD_CYCLES_VALU", 0) / max(1, agg["SQ_ACTIVE_INST_VALU"]) / 64, 3))
