#!/bin/bash
# r05b: the drop-in rebuilt around one staged feed (pusher / film threads, copy-engine snapshots, cost tail):
# its GPU tests, the production parity suite (the kernel gained the staged feed's per-tile job counts and the
# fetch's acquire), then the drain sweep with a feed trace of one C3 frame.
set -eu
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_integration.py \
  > $O/pytest_integration.log 2>&1 || { tail -30 $O/pytest_integration.log; exit 1; }
tail -3 $O/pytest_integration.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_production.py \
  > $O/pytest_production.log 2>&1 || { tail -30 $O/pytest_production.log; exit 1; }
tail -2 $O/pytest_production.log
bash tools/drain_sweep.sh $O/drain
VPT_FEED_TRACE=1 timeout -k 10 120 tests/native/build/run_gpu_harness config=volume_path_tracer_amd/scenes/wdas_cloud.json \
  out=$O/film.f32 w=1920 h=1080 waves=256 grid_n=512 threads=1 batch=4096 > $O/trace_c3.log 2>&1
rm -f $O/film.f32
grep -v "slotwait" $O/trace_c3.log | tail -25
