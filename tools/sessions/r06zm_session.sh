#!/bin/bash
# r06zm: C4 on gate_idle 1, short: production parity and the C4 bench line.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06zm; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_production.py -x -q --timeout 120 --timeout-method thread > $O/pytest_production.log 2>&1 || { tail -20 $O/pytest_production.log; exit 1; }
tail -1 $O/pytest_production.log
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --cpu-budget 6 > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench_c4.json').read().strip().splitlines()[-1]); x=d['dropin']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity'].get('bit_identical'), x.get('ms_frames'), x.get('bit_identical_to_one_launch'), x['first_call'].get('total_ms'))"
