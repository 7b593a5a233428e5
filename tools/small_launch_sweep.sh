#!/bin/bash
# Grid sizes for C2's partly filled launch (262 144 jobs) and latency gates for C1 (4 096 jobs).
set -u
export TMPDIR=/tmp; O=gpurun_out/${1:-small}; mkdir -p $O
timeout -k 10 300 python tools/tune.py --config c2 --spp 64 --gates 6:8:36:4 --blocks ${C2BLOCKS:-512,640,768,1024,1280} --reps 2 > $O/c2.log 2>&1 || { tail -5 $O/c2.log; exit 1; }
grep Msps $O/c2.log | grep -o '"lat".*'
[ -n "${NOC1:-}" ] || timeout -k 10 300 python tools/tune.py --config c1 --spp 4 --gates 6:8:36:4 --blocks 1792 --lat 0:1:65:1:1,0:1:65:2:1,0:1:65:1:2,0:1:65:4:1,0:1:65:1:4,0:2:65:1:1 --reps 3 > $O/c1.log 2>&1 || { tail -5 $O/c1.log; exit 1; }
[ -n "${NOC1:-}" ] || grep Msps $O/c1.log | grep -o '"lat".*'
