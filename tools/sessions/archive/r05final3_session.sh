#!/bin/bash
# r05final3: the round's last GPU check on the final code: C4 PMC passes + kernel trace (its gate default changed),
# the whole GPU suite and smoke, bench.py C3 (drop-in, CPU baseline, parity) and C4 / C2 / C1 / C5 lines.
set -u
O=gpurun_out/r05final3; mkdir -p $O
bash tools/profile_round.sh r05final3 c4 || exit 1
STEPS="pytest smoke bench" bash tools/gpu_check.sh r05final3 || exit 1
for c in c4 c2 c1; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || { tail -5 $O/bench_$c.log; exit 1; }
  tail -1 $O/bench_$c.log | cut -c1-300
done
timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log | cut -c1-300
echo "all steps done"
