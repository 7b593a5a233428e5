#!/bin/bash
# GPU parity tests on the default library, then A/B timing of library builds on one box
# (full C3 frame at the default gates).  Usage: LIBS="libvpt_amd_base libvpt_amd" bash tools/ab.sh <tag>
export TMPDIR=/tmp; O=gpurun_out/${1:-ab}; mkdir -p $O
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
fi
for L in ${LIBS:-libvpt_amd_base libvpt_amd}; do
  for OR in ${ORDERS:--1}; do
    VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 300 python tools/tune.py --config ${CONFIG:-c3} --spp ${SPP:-256} --gates ${GATES:-8:12:32:4} --reps ${REPS:-3} --order $OR > $O/$L.o$OR.log 2>&1 || exit $?
    echo "$L order=$OR $(grep Msps $O/$L.o$OR.log | tail -1 | cut -c1-200)"
  done
done
