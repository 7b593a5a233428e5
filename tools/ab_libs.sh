#!/bin/bash
# A/B of library builds on one GPU box: GPU parity tests against each experimental library (VPT_LIB),
# then timing of the full C3 frame (tools/tune.py, default gates) for each, alternating.
# Usage: LIBS="libvpt_amd libvpt_amd_x" [TESTS="tests/test_gpu_production.py"] bash tools/ab_libs.sh <tag> [tune args]
set -u
export TMPDIR=/tmp; O=gpurun_out/${1:-ab}; shift || true; mkdir -p $O
for L in ${LIBS}; do
  if [ -n "${TESTS:-}" ]; then
    VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 600 python -u -m pytest ${TESTS} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_$L.log 2>&1
    rc=$?; echo "$L pytest rc=$rc $(tail -1 $O/pytest_$L.log)"; if [ $rc -ne 0 ]; then exit $rc; fi
  fi
done
for R in ${ROUNDS:-1 2}; do
  for L in ${LIBS}; do
    VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 300 python tools/tune.py --config ${CONFIG:-c3} --spp ${SPP:-256} --gates ${GATES:-6:8:36:4} --reps ${REPS:-2} "$@" > $O/$L.r$R.log 2>&1
    rc=$?; echo "$L round $R rc=$rc $(grep Msps $O/$L.r$R.log | tail -1 | grep -o '"ms".*')"; if [ $rc -ne 0 ]; then tail -3 $O/$L.r$R.log; exit $rc; fi
  done
done
