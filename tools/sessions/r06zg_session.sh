#!/bin/bash
# r06zg: the ordered-film / job-order GPU tests (with the full-launch same-tile test), then the walk gate of the temperature kernel under the same-tile order (r06zf: C4 8:8:36:2 69.1 ms vs 71.2 at
# the default 8:8:36:4) and C3's gate_min 4 (321.1 vs 321.8), re-swept twice each with best-of-3 full frames.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06zg; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_film_order.py tests/test_gpu_order.py -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_order.log 2>&1 || { tail -20 $O/pytest_order.log; exit 1; }
tail -1 $O/pytest_order.log
G4="8:8:36:4,8:8:36:2,8:8:36:1,8:8:36:3,10:8:36:2,8:8:28:2,10:8:28:2,6:8:36:2"
G3="6:8:36:4,4:8:36:4,6:8:36:3,4:8:36:3,6:8:36:2"
for r in 1 2; do
  timeout -k 10 300 python tools/tune.py --config c4 --spp 256 --gates $G4 --reps 3 > $O/gates_c4_$r.jsonl 2> $O/gates_c4_$r.err || { tail -5 $O/gates_c4_$r.err; exit 1; }
  timeout -k 10 300 python tools/tune.py --config c3 --spp 256 --gates $G3 --reps 3 > $O/gates_c3_$r.jsonl 2> $O/gates_c3_$r.err || { tail -5 $O/gates_c3_$r.err; exit 1; }
done
python3 -c "
import json
for c in ('c3', 'c4'):
    rows = {}
    for r in (1, 2):
        for l in open('$O/gates_%s_%d.jsonl' % (c, r)):
            d = json.loads(l); rows.setdefault(d['gate'], []).append(d['ms'])
    for g, v in rows.items(): print(c, g, v)
" | tee $O/summary.txt
