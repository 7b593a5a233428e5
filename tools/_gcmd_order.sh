#!/bin/bash
# Job-order A/B: GPU order tests, then modes 0/1/2 at several spp on the full C3 frame.
export TMPDIR=/tmp; O=gpurun_out/order; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "order or edge" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for S in ${SPPS:-32 256 512}; do for OR in ${ORDERS:-0 1 2}; do
  timeout -k 10 300 python tools/tune.py --spp $S --gates 8:12:24:4 --reps 2 --order $OR > $O/s$S.o$OR.log 2>&1 || exit $?
  echo "spp=$S order=$OR $(grep Msps $O/s$S.o$OR.log | tail -1 | cut -c1-200)"
done; done
