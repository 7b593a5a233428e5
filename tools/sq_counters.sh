#!/bin/bash
# SQ / TCP / TCC counters of one C3 bench step (rocprofv3 --pmc, one pass per group, each under its own
# time limit).  Usage (GPU box): bash tools/sq_counters.sh <outdir> [bench args, e.g. --spp 64]
set -u
O=${1:-gpurun_out/sq}; shift || true; mkdir -p $O; export TMPDIR=/tmp
PASSES=${PASSES:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT
TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum"}
i=0
while IFS= read -r P; do
  [ -z "$P" ] && continue
  i=$((i+1)); N=p$i
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$N -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-dropin "$@" > $O/pmc_$N.log 2>&1
  rc=$?; echo "pass $i ($P) rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $O/pmc_$N.log; exit $rc; fi
done <<< "$PASSES"
