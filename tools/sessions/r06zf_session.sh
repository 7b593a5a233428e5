#!/bin/bash
# r06zf: the whole GPU suite and smoke with the same-tile order on full launches only; C2 and the C3 8-GPU share
# (partly filled launches, back on the cost tail) and the C3 frame; then the full-occupancy gates re-swept under the
# same-tile order (C3 / C4 full frames, gate_min:gate_idle:gate_eval:gate_walk around the defaults).
set -u
export TMPDIR=/tmp
O=gpurun_out/r06zf; mkdir -p $O
STEPS="pytest smoke" bash tools/gpu_check.sh r06zf || exit $?
grep -E "passed|failed" $O/pytest_gpu.log | tail -1
for spec in "c2 64" "c3 32" "c3 256"; do
  set -- $spec
  timeout -k 10 200 python bench.py --config $1 --spp $2 --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/b_$1_$2.json 2> $O/b_$1_$2.err || exit 1
  echo "$1 spp $2 $(grep -o '"ms_per_step": [0-9.]*' $O/b_$1_$2.json)" | tee -a $O/summary.txt
done
G3="6:8:36:4,4:8:36:4,8:8:36:4,6:12:36:4,6:8:28:4,6:8:44:4,6:8:36:2,6:8:36:6"
G4="8:8:36:4,6:8:36:4,10:8:36:4,8:12:36:4,8:8:28:4,8:8:44:4,8:8:36:2,8:8:36:6"
timeout -k 10 400 python tools/tune.py --config c3 --spp 256 --gates $G3 --reps 2 > $O/gates_c3.jsonl 2> $O/gates_c3.err || { tail -5 $O/gates_c3.err; exit 1; }
timeout -k 10 400 python tools/tune.py --config c4 --spp 256 --gates $G4 --reps 2 > $O/gates_c4.jsonl 2> $O/gates_c4.err || { tail -5 $O/gates_c4.err; exit 1; }
python3 -c "
import json
for c in ('c3', 'c4'):
    for l in open('$O/gates_%s.jsonl' % c):
        d = json.loads(l); print(c, d['gate'], d['ms'])
"
