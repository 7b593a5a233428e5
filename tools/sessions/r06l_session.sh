#!/bin/bash
# r06l: run()'s phases with the helper-thread overlap and the two grids flattened side by side (first_call, C3 / C4),
# and the GPU integration + film-order suites on that code (SESSION=r06m: the host grids released on a thread of
# their own; r06n: huge pages; r06o: the flatten beside the HIP start, vpt_grids_flatten + vpt_gpu_create_from;
# r06p: the host grids released beside the frame; r06q: kept until the next run() or exit).
set -u
export TMPDIR=/tmp
O=gpurun_out/${SESSION:-r06l}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_integration.py tests/test_gpu_film_order.py -x -q --timeout 120 --timeout-method thread > $O/pytest_integration.log 2>&1 || { tail -30 $O/pytest_integration.log; exit 1; }
tail -2 $O/pytest_integration.log
for C in c4 c3; do
  timeout -k 10 300 python bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --dropin-frames 1 > $O/bench_$C.json 2> $O/bench_$C.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$C.json').read().strip().splitlines()[-1]); print('$C', d['ms_per_step'], d['dropin'].get('first_call'))"
done
