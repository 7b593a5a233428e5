#!/bin/bash
# r05gates: the wave gates re-swept on the final kernels (the film regroup changed what the finish pass costs):
# C4 and C3 at 256 spp, best of 2 per setting, the default 6:8:36:4 first and last (drift check).
set -u
O=gpurun_out/r05gates; mkdir -p $O
G=6:8:36:4,4:8:36:4,8:8:36:4,12:8:36:4,6:8:24:4,6:8:48:4,6:4:36:4,6:16:36:4,6:8:36:2,6:8:36:8,6:8:36:4
for c in c4 c3; do
  timeout -k 10 600 python tools/tune.py --config $c --spp 256 --gates $G --reps 2 > $O/$c.jsonl 2>&1 || { tail -5 $O/$c.jsonl; exit 1; }
  python3 -c "
import json,sys
for l in open('$O/$c.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$c', d['gate'], d['ms'])
"
done
echo "all steps done"
