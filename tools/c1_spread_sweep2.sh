#!/bin/bash
# C1 frames of 16 / 32 / 48 spp on the full grid: job lanes per wavefront 1 / 2 / 3 / auto.
set -u
export TMPDIR=/tmp; O=gpurun_out/${1:-c1s2}; mkdir -p $O
for S in 16 32 48; do
  timeout -k 10 300 python tools/tune.py --config c1 --spp $S --gates 6:8:36:4 --blocks 1792 --lat 1:1:65:1:1,2:1:65:1:1,3:1:65:1:1,0:1:65:1:1 --reps 2 > $O/c1_$S.log 2>&1 || { tail -5 $O/c1_$S.log; exit 1; }
  grep Msps $O/c1_$S.log | grep -o '"lat".*'
done
