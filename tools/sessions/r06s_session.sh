#!/bin/bash
# r06s: the drop-in's ordered frame (run()'s film in wave order, bit-identical): the GPU integration suite, then C4 /
# C3 bench lines whose drop-in frames run ordered and are compared bit for bit with the one-launch frame.
set -u
export TMPDIR=/tmp
O=gpurun_out/${SESSION:-r06s}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_integration.py -x -v --timeout 120 --timeout-method thread > $O/pytest_integration.log 2>&1 || { tail -40 $O/pytest_integration.log; exit 1; }
grep -E "passed|failed" $O/pytest_integration.log | tail -1
for C in c4 c3; do
  timeout -k 10 400 python bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --dropin-frames 3 > $O/bench_$C.json 2> $O/bench_$C.err || { tail -20 $O/bench_$C.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$C.json').read().strip().splitlines()[-1]); x=d['dropin']; print('$C', d['ms_per_step'], {k: x.get(k) for k in ['ms_frames','bit_identical_to_one_launch','pixels_differing_from_one_launch','provider_alone_ms']}, x['first_call'].get('total_ms'), x['first_call'].get('frame_ms'))"
done
