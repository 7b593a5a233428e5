#!/bin/bash
# r06zi: the round's closing check on the committed tree: the whole GPU suite and smoke, then the default bench
# line exactly as the driver runs it (C3; its roofline inputs from the committed r06zd profiles).
set -u
export TMPDIR=/tmp
STEPS="pytest smoke" bash tools/gpu_check.sh r06zi || exit $?
grep -E "passed|failed" gpurun_out/r06zi/pytest_gpu.log | tail -1
timeout -k 10 600 python bench.py > gpurun_out/r06zi/bench_c3.json 2> gpurun_out/r06zi/bench_c3.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r06zi/bench_c3.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['traffic_source'], r.get('request_sources'), d['parity'].get('bit_identical'), d['dropin'].get('ms_frames'), d['dropin'].get('bit_identical_to_one_launch'))"
