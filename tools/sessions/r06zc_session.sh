#!/bin/bash
# r06zc: the same-tile job order re-measured on the ordered film (r03 measured it against the film atomics, whose
# 64 lanes adding to one pixel at once serialised): C3 / C4 full frames, default order vs same-tile, alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06zc; mkdir -p $O
for r in 1 2; do
  for c in c3 c4; do
    for p in "" same-tile; do
      timeout -k 10 300 python tools/tune.py --config $c --spp 256 --gates $([ $c = c4 ] && echo 8:8:36:4 || echo 6:8:36:4) --reps 3 ${p:+--perm $p} >> $O/tune.jsonl 2> $O/tune_${c}_${r}.err || { tail -5 $O/tune_${c}_${r}.err; exit 1; }
      tail -1 $O/tune.jsonl
    done
  done
done
