#!/bin/bash
# r06zj: C4's other gates around the new walk gate 1 (gate_min, gate_idle, gate_eval), best of 3 full frames, twice.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06zj; mkdir -p $O
G4="8:8:36:1,10:8:36:1,12:8:36:1,8:8:28:1,8:8:44:1,8:12:36:1,8:4:36:1,8:8:36:0"
for r in 1 2; do
  timeout -k 10 300 python tools/tune.py --config c4 --spp 256 --gates $G4 --reps 3 > $O/gates_c4_$r.jsonl 2> $O/gates_c4_$r.err || { tail -5 $O/gates_c4_$r.err; exit 1; }
done
python3 -c "
import json
rows = {}
for r in (1, 2):
    for l in open('$O/gates_c4_%d.jsonl' % r):
        d = json.loads(l); rows.setdefault(d['gate'], []).append(d['ms'])
for g, v in rows.items(): print('c4', g, v)
" | tee $O/summary.txt
