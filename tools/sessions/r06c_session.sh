#!/bin/bash
# r06c: the mock taker rate over batch sizes / devices on the box's cores; the rest of the integration tests;
# then the default bench lines (C3, C4) with first_call and the bit-identical parity.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06c; mkdir -p $O
M=tests/native/build/dropin_mock_rate
for b in 4096 16384 65536; do for d in 1 2 8; do for i in 1 2 3; do
  timeout -k 5 60 $M multi=1 devices=$d cheap=1 rate=1 w=1920 h=1080 waves=64 batch=$b blocks=1792 threads=256 | grep rate | sed "s/^/batch $b devices $d: /" >> $O/mock_rate.txt || exit 1
done; done; done
cat $O/mock_rate.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_integration.py -x -v -s -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "not mock_taker_rate" > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|rewritten" $O/pytest.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
cut -c1-300 $O/bench_c3.json
timeout -k 10 600 python bench.py --config c4 > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
cut -c1-300 $O/bench_c4.json
