#!/bin/bash
# Round-end check on one box: every GPU test, smoke, the C1 / C2 / C4 config bench lines and the
# default (C3) bench.  Stops at the first failing step.
set -u
export TMPDIR=/tmp; O=gpurun_out/${1:-final}; mkdir -p $O
STEPS="pytest smoke" bash tools/gpu_check.sh ${1:-final}/check || exit $?
grep -q "passed" $O/check/pytest_gpu.log && ! grep -q "failed" $O/check/pytest_gpu.log || { echo "pytest failed"; tail -20 $O/check/pytest_gpu.log; exit 1; }
grep -q "smoke ok" $O/check/smoke.log || { echo "smoke failed"; exit 1; }
for C in c1 c2 c4; do
  timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --cpu-budget 6 > $O/bench_$C.json 2> $O/bench_$C.err || exit 1
  cut -c1-300 $O/bench_$C.json
done
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
cut -c1-300 $O/bench_c3.json
