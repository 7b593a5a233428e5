"""Summarise tools/sq_counters.sh output: python tools/sq_summary.py <outdir> [samples]
SQ cycle counters count quad-cycles (MI355X_MICROARCH.md); ratios between them are unit-free."""
import collections
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
samples = float(sys.argv[2]) if len(sys.argv) > 2 else 1920 * 1080 * 64
agg = collections.defaultdict(float)
for f in d.rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "integrate" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(agg):
    print(f"{k:30s} {agg[k]:18.4g}   per sample {agg[k] / samples:10.3f}")
g = agg.get
if g("SQ_WAVE_CYCLES"):
    wc = agg["SQ_WAVE_CYCLES"]
    print("VALU active / wave cycles   ", round(g("SQ_ACTIVE_INST_VALU", 0) / wc, 3))
    print("any inst active / wave cyc  ", round(g("SQ_ACTIVE_INST_ANY", 0) / wc, 3))
    print("wait_any / wave cycles      ", round(g("SQ_WAIT_ANY", 0) / wc, 3))
    print("wait_inst_any / wave cycles ", round(g("SQ_WAIT_INST_ANY", 0) / wc, 3))
    if g("SQ_ACTIVE_INST_VALU"):
        print("VALU lane utilisation       ", round(g("SQ_THREAD_CYCLES_VALU", 0) / agg["SQ_ACTIVE_INST_VALU"] / 64, 3))
if g("SQ_BUSY_CYCLES") and g("SQ_ACTIVE_INST_VALU"):
    print("VALU active per SIMD-busy (waves summed) ", round(agg["SQ_ACTIVE_INST_VALU"] / agg["SQ_BUSY_CYCLES"], 3))
if g("TCC_HIT_sum"):
    print("L2 hit rate                 ", round(agg["TCC_HIT_sum"] / (agg["TCC_HIT_sum"] + g("TCC_MISS_sum", 0)), 3))
if g("TCP_TOTAL_CACHE_ACCESSES_sum"):
    print("L1 -> L2 read requests / L1 accesses", round(g("TCP_TCC_READ_REQ_sum", 0) / agg["TCP_TOTAL_CACHE_ACCESSES_sum"], 3))
