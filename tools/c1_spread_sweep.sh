#!/bin/bash
# C1 (4 096 jobs): grid size with exactly one job lane per wavefront (wave_lanes 1) vs the auto choice.
set -u
export TMPDIR=/tmp; O=gpurun_out/${1:-c1s}; mkdir -p $O
timeout -k 10 300 python tools/tune.py --config c1 --spp 4 --gates 6:8:36:4 --blocks 1024,1280,1536,1792 --lat 1:1:65:1:1,2:1:65:1:1 --reps 3 > $O/c1.log 2>&1 || { tail -5 $O/c1.log; exit 1; }
grep Msps $O/c1.log | grep -o '"lat".*'
timeout -k 10 300 python tools/tune.py --config c1 --spp 8 --gates 6:8:36:4 --blocks 1792 --lat 1:1:65:1:1,2:1:65:1:1,3:1:65:1:1 --reps 3 > $O/c1_8.log 2>&1 || { tail -5 $O/c1_8.log; exit 1; }
grep Msps $O/c1_8.log | grep -o '"lat".*'
