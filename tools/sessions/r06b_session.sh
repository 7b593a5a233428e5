#!/bin/bash
# r06b: the single-taker multi-context drop-in, the GPU seed search, the mock taker rate on the box's cores;
# then the full default bench lines (C3, C4) with the drop-in's first_call record and the bit-identical parity.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_integration.py -x -v -s -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|rate|seed .* ms" $O/pytest.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
cut -c1-300 $O/bench_c3.json
timeout -k 10 600 python bench.py --config c4 > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
cut -c1-300 $O/bench_c4.json
