#!/bin/bash
# r05g: live-path compaction on the latency kernel: its bit-exactness tests, then C2 frames
# without / with compaction every 1 / 2 / 4 / 8 / 16 / 32 outer iterations (tools/tune.py, the exchange count
# per run), then the SQ counters of C2 without and with the best period.
set -u
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_production.py \
  -k "compacting" > $O/pytest_compact.log 2>&1 || { tail -30 $O/pytest_compact.log; exit 1; }
tail -2 $O/pytest_compact.log
timeout -k 10 600 python tools/tune.py --config c2 --spp 64 --gates 6:8:36:4 --blocks 512 --lat-kernel 1 --lat-ungated 0 \
  --compact 0,1,2,4,8,16,32,0 --reps 3 > $O/c2_compact.jsonl 2> $O/c2_compact.err || { tail $O/c2_compact.err; exit 1; }
cat $O/c2_compact.jsonl
