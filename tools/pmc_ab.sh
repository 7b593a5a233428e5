#!/bin/bash
# One SQ counter pass per library build (same counters), for instruction-mix A/B.
# Usage (GPU box): LIBS="libvpt_amd libvpt_amd_x" bash tools/pmc_ab.sh <tag> [bench args]
set -u
O=gpurun_out/${1:-pmcab}; shift || true; mkdir -p $O; export TMPDIR=/tmp
P=${PMC:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_THREAD_CYCLES_VALU"}
for L in ${LIBS}; do
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/$L -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $O/$L.log 2>&1
  rc=$?; echo "$L rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $O/$L.log; exit $rc; fi
done
