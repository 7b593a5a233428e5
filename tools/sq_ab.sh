#!/bin/bash
# SQ counter pass (one C3 launch) per library build, for A/B attribution of a timing difference.
# Usage (GPU box): LIBS="libvpt_amd libvpt_amd_x" bash tools/sq_ab.sh <outdir>
set -u
O=${1:-gpurun_out/sqab}; mkdir -p $O; export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM"
for L in ${LIBS}; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/$L/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-dropin > $O/$L.p$i.log 2>&1
    rc=$?; echo "$L pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $O/$L.p$i.log; exit $rc; fi
  done
done
