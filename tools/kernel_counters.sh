#!/bin/bash
# Kernel-level counters of one integrator launch for profiles/: SQ (waves, waits, VALU lane use,
# instruction mix, memory in flight) and the vector-memory pipeline (TA / TD busy and stalls, TCP
# pending stalls, L1->L2 read requests and their latency), one rocprofv3 --pmc pass per group, each
# under its own time limit; then tools/kernel_counters.py writes gpurun_out/<tag>_<config>/counters.json.
# Usage (GPU box): bash tools/kernel_counters.sh <tag> [config] [bench args...]
set -u
TAG=${1:-r03}; CFG=${2:-c3}; shift 2 || shift $#
O=gpurun_out/${TAG}_${CFG}_counters; mkdir -p $O; export TMPDIR=/tmp
i=0
while IFS= read -r P; do
  [ -z "$P" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/pass_$i -o run -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-dropin "$@" > $O/pass_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc: $P"; if [ $rc -ne 0 ]; then tail -3 $O/pass_$i.log; exit $rc; fi
done <<'PASSES'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
PASSES
python3 tools/kernel_counters.py $O $CFG "$@" > $O/summary.txt && cat $O/summary.txt | tail -25
