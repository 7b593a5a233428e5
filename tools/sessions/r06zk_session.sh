#!/bin/bash
# r06zk: C4 on gate_idle 4 (r06zj): production parity, its roofline inputs and bench line; then gate_idle re-swept
# for both kernels on the same-tile order.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06zk; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_production.py -x -q --timeout 120 --timeout-method thread > $O/pytest_production.log 2>&1 || { tail -20 $O/pytest_production.log; exit 1; }
tail -1 $O/pytest_production.log
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --cpu-budget 6 > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench_c4.json').read().strip().splitlines()[-1]); x=d['dropin']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity'].get('bit_identical'), x.get('ms_frames'), x.get('bit_identical_to_one_launch'), x['first_call'].get('total_ms'))"
timeout -k 10 300 python tools/tune.py --config c4 --spp 256 --gates 8:4:36:1,8:2:36:1,8:1:36:1,8:4:28:1,8:4:36:2 --reps 3 > $O/gates_c4.jsonl 2> $O/gates_c4.err || { tail -5 $O/gates_c4.err; exit 1; }
timeout -k 10 300 python tools/tune.py --config c3 --spp 256 --gates 6:8:36:4,6:4:36:4,6:2:36:4,6:4:36:2 --reps 3 > $O/gates_c3.jsonl 2> $O/gates_c3.err || { tail -5 $O/gates_c3.err; exit 1; }
python3 -c "
import json
for c in ('c4', 'c3'):
    for l in open('$O/gates_%s.jsonl' % c):
        d = json.loads(l); print(c, d['gate'], d['ms'])
" | tee $O/summary.txt
bash tools/profile_round.sh r06zk c4 || exit $?
bash tools/kernel_counters.sh r06zk c4 || exit $?
