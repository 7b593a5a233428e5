#!/bin/bash
# SQ instruction-mix / busy counters of one C3 bench step (rocprofv3 --pmc, one pass per group).
# Usage (GPU box): bash tools/sq_counters.sh <outdir> [bench args]
set -u
O=${1:-gpurun_out/sq}; shift || true; mkdir -p $O; export TMPDIR=/tmp
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH" "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32" "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD"; do
  N=$(echo $P | cut -d' ' -f1-2 | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$N -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $O/pmc_$N.log 2>&1
  rc=$?; echo "$P rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $O/pmc_$N.log; exit $rc; fi
done
