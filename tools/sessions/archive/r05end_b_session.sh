#!/bin/bash
# r05end (b): C4 PMC passes + kernel trace (tools/profile_round.sh), then the C4 / C2 / C1 bench lines, the whole GPU
# suite and smoke.
set -u
bash tools/profile_round.sh r05end c4 || exit 1
for c in c4 c2 c1; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > gpurun_out/r05end_c4/bench_$c.log 2>&1 || { tail -5 gpurun_out/r05end_c4/bench_$c.log; exit 1; }
  tail -1 gpurun_out/r05end_c4/bench_$c.log | cut -c1-300
done
STEPS="pytest smoke" bash tools/gpu_check.sh r05end || exit 1
echo "all steps done"
