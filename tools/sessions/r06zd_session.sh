#!/bin/bash
# r06zd: the roofline inputs on the final binary (full-rate table indexes, the same-tile job order): PMC traffic +
# kernel trace and the C3 bench line, kernel counter passes, for C3 and C4, and C4's bench line (the GPU suite and
# smoke on this binary: r06zf).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06zd
bash tools/profile_round.sh r06zd c3 || exit $?
bash tools/profile_round.sh r06zd c4 || exit $?
bash tools/kernel_counters.sh r06zd c3 || exit $?
bash tools/kernel_counters.sh r06zd c4 || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --cpu-budget 6 > gpurun_out/r06zd/bench_c4.json 2> gpurun_out/r06zd/bench_c4.err || exit 1
for f in gpurun_out/r06zd_c3/bench.log gpurun_out/r06zd/bench_c4.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); x=d['dropin']; print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity'].get('bit_identical'), {k: x.get(k) for k in ['ms_frames','bit_identical_to_one_launch']}, x['first_call'].get('total_ms'))"; done
