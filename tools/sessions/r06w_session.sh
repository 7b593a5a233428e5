#!/bin/bash
# r06w: the whole GPU suite and smoke on the code with run()'s ordered frame, then the default bench line (C3:
# its drop-in frame compared bit for bit with the one-launch frame) and C4's.
set -u
export TMPDIR=/tmp
STEPS="pytest smoke" bash tools/gpu_check.sh r06w || exit $?
grep -E "passed|failed" gpurun_out/r06w/pytest_gpu.log | tail -1
timeout -k 10 600 python bench.py > gpurun_out/r06w/bench_c3.json 2> gpurun_out/r06w/bench_c3.err || exit 1
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 --cpu-budget 6 > gpurun_out/r06w/bench_c4.json 2> gpurun_out/r06w/bench_c4.err || exit 1
for C in c3 c4; do python3 -c "import json; d=json.loads(open('gpurun_out/r06w/bench_$C.json').read().strip().splitlines()[-1]); x=d['dropin']; print('$C', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity'].get('bit_identical'), {k: x.get(k) for k in ['ms_frames','bit_identical_to_one_launch','pixels_differing_from_one_launch']}, x['first_call'].get('total_ms'))"; done
