#!/bin/bash
# r05j: split launches (vpt_gpu_set_split) for partly filled frames -- the costliest tiles' jobs on CUs of
# their own: their bit-exactness tests, then the C3 8-GPU share (32 waves) across CU counts / tile fractions.
set -u
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_production.py \
  -k "split" > $O/pytest_split.log 2>&1 || { tail -30 $O/pytest_split.log; exit 1; }
tail -2 $O/pytest_split.log
timeout -k 10 600 python tools/tune.py --config c3 --spp 32 --gates 6:8:36:4 --reps 3 \
  --split 0:0:0,16:0.01:2,32:0.01:2,32:0.02:2,32:0.04:2,48:0.03:2,64:0.05:2,32:0.02:1,32:0.02:4,0:0:0 \
  > $O/c3s32_split.jsonl 2> $O/c3s32_split.err || { tail $O/c3s32_split.err; exit 1; }
cut -c1-60,150-400 $O/c3s32_split.jsonl
