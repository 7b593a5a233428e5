#!/bin/bash
# r05o: the whole GPU suite and smoke on the round's code (NUMA-bound pusher, film-thread schedule), then
# bench.py C3 (its dropin record, CPU baseline) and C4 / C2 / C1 lines.
set -u
STEPS="pytest smoke bench" bash tools/gpu_check.sh r05o || exit 1
for c in c4 c2 c1; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > gpurun_out/r05o/bench_$c.log 2>&1 || { tail -5 gpurun_out/r05o/bench_$c.log; exit 1; }
  tail -1 gpurun_out/r05o/bench_$c.log | cut -c1-300
done
