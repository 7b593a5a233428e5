#!/bin/bash
# r05gates2: C4's gate_min 8 vs 6 (r05gates: 84.0 vs 84.8-85.0 once), 4 alternating runs of each, best of 3.
set -u
O=gpurun_out/r05gates2; mkdir -p $O
for r in 1 2 3 4; do
  for g in 6:8:36:4 8:8:36:4; do
    timeout -k 10 300 python tools/tune.py --config c4 --spp 256 --gates $g --reps 3 > $O/c4_${g//:/_}_$r.jsonl 2>&1 || exit 1
    echo "c4 round $r $g $(grep -o '"ms": [0-9.]*' $O/c4_${g//:/_}_$r.jsonl)"
  done
done
echo "all steps done"
