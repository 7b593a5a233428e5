"""Summarise tools/kernel_counters.sh passes into <outdir>/counters.json (one integrator launch).

Per-CU counters (*_sum) are summed over the 256 CUs; GRBM_GUI_ACTIVE is the GPU's busy clock summed
over the 8 XCDs (cycles per CU = GRBM_GUI_ACTIVE / 8 over the launch).  SQ cycle counters count
quad-cycles (MI355X_MICROARCH.md); only their ratios are used.  Samples per launch = the bench
line's width x height x spp (one step at N = 1, which bench.py checks against the kernel's count).
Usage: python tools/kernel_counters.py <outdir> <config>"""
import csv
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

d, config = Path(sys.argv[1]), sys.argv[2]
bench_args = sys.argv[3:]  # extra bench.py arguments of the passes (e.g. --grid-n 384: not the config's workload)
if os.environ.get("VPT_LIB"):  # a variant library (an experiment): not the production kernel's counters
    bench_args = bench_args + ["VPT_LIB=" + os.path.basename(os.environ["VPT_LIB"])]
vals = defaultdict(list)
ms = []
samples = None
for p in sorted(d.glob("pass_*")):
    if p.is_dir():
        per = defaultdict(float)
        for f in p.rglob("*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                if "integrate" in r["Kernel_Name"]:
                    per[r["Counter_Name"]] += float(r["Counter_Value"])
        for k, v in per.items():
            vals[k].append(v)
    elif p.suffix == ".log":
        for line in p.read_text().splitlines():
            if line.startswith("{") and '"metric"' in line:
                j = json.loads(line)
                ms.append(j["roofline"]["avg_launch_ms"])
                cfg = j["config"]
                samples = cfg["width"] * cfg["height"] * cfg["spp"]  # the one timed step (N = 1)
c = {k: sum(v) / len(v) for k, v in vals.items()}
g = c.get
cus = 256
cycles = g("GRBM_GUI_ACTIVE", 0) / 8.0  # per XCD = per CU
der = {}
if samples:
    der["l1_to_l2_requests_per_sample"] = g("TCP_TCC_READ_REQ_sum", 0) / samples
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM", "SQ_INSTS_LDS",
              "SQ_INSTS_BRANCH", "SQ_WAIT_ANY"):
        if g(k) is not None:
            der[k.lower() + "_per_sample"] = g(k) / samples
if cycles:
    der["cycles_per_cu"] = cycles
    for k, n in (("TA_TA_BUSY_sum", "ta_busy"), ("TA_ADDR_STALLED_BY_TC_CYCLES_sum", "ta_addr_stalled_by_tcp"),
                 ("TD_TD_BUSY_sum", "td_busy"), ("TD_TC_STALL_sum", "td_stalled_by_tcp"),
                 ("TCP_PENDING_STALL_CYCLES_sum", "tcp_pending_stall")):
        if g(k) is not None:
            der[n] = g(k) / cus / cycles
if g("TCP_TCC_READ_REQ_sum"):
    der["l2_read_latency_cycles"] = g("TCP_TCC_READ_REQ_LATENCY_sum", 0) / g("TCP_TCC_READ_REQ_sum")
    if g("TCP_TOTAL_CACHE_ACCESSES_sum"):
        der["l1_hit_rate"] = 1.0 - g("TCP_TCC_READ_REQ_sum") / g("TCP_TOTAL_CACHE_ACCESSES_sum")
    if ms:
        der["l1_to_l2_requests_per_s_per_cu"] = g("TCP_TCC_READ_REQ_sum") / (sum(ms) / len(ms) / 1e3) / cus
if g("SQ_WAVE_CYCLES"):
    wc = g("SQ_WAVE_CYCLES")
    der["valu_active_per_wave_cycle"] = g("SQ_ACTIVE_INST_VALU", 0) / wc
    der["wait_any_per_wave_cycle"] = g("SQ_WAIT_ANY", 0) / wc
    der["issue_any_per_wave_cycle"] = g("SQ_ACTIVE_INST_ANY", 0) / wc
    if g("SQ_ACTIVE_INST_VALU"):
        der["valu_lane_utilisation"] = g("SQ_THREAD_CYCLES_VALU", 0) / g("SQ_ACTIVE_INST_VALU") / 64
if g("SQ_INST_LEVEL_VMEM") and g("SQ_INSTS_VMEM_RD"):
    der["vmem_in_flight_per_instruction"] = g("SQ_INST_LEVEL_VMEM") / (g("SQ_INSTS_VMEM_RD") + g("SQ_INSTS_VMEM_WR", 0))
out = {"config": config, "bench_args": bench_args, "kernel": "vpt_integrate_kernel", "samples_per_launch": samples,
       "kernel_ms_per_pass": ms, "counters_per_launch": {k: round(v, 1) for k, v in sorted(c.items())},
       "derived": {k: round(v, 6) for k, v in der.items()},
       "method": "rocprofv3 --pmc, one pass per counter group (tools/kernel_counters.sh), one launch of "
                 "bench.py --steps 1 --warmup 0; *_sum summed over 256 CUs; GRBM_GUI_ACTIVE / 8 = cycles per CU"}
(d / "counters.json").write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out, indent=1))
