#!/bin/bash
# r06d: the pusher over runs (no per-job division): the mock taker rate on the box's cores at 1 / 2 / 8 mock
# GPUs, the drop-in integration tests, then the C4 and C3 drop-in frames (bench dropin + first_call).
set -u
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
M=tests/native/build/dropin_mock_rate
for d in 1 2 8; do for i in 1 2 3; do
  timeout -k 5 60 $M multi=1 devices=$d cheap=1 rate=1 w=1920 h=1080 waves=64 batch=4096 blocks=1792 threads=256 | grep -E "rate|provider alone" | sed "s/^/devices $d: /" >> $O/mock_rate.txt || exit 1
done; done
cat $O/mock_rate.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_integration.py -x -v -s -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|rewritten|x\)" $O/pytest.log | tail -8
for C in c4 c3; do
  timeout -k 10 600 python bench.py --config $C --steps 3 --no-cpu-baseline > $O/bench_$C.json 2> $O/bench_$C.err || exit 1
  python -c "import json,sys; j=json.load(open('$O/bench_$C.json')); d=j.get('dropin',{}); print('$C', j['ms_per_step'], d.get('ms_frames'), d.get('provider_alone_ms'), {k: d.get('first_call',{}).get(k) for k in ('total_ms','seed_ms','contexts_ms','flatten_fix_ms','upload_ms','tile_costs_ms','frame_ms','hip_ms')})"
done
exit $rc
