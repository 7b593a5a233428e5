#!/bin/bash
# r05d: the drop-in after the overhead trims (feed-owned stream, clean-ring reuse, clear overlapped with the
# final add): integration tests, the drain sweep, and C3 / C4 feed traces.
set -eu
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_integration.py \
  > $O/pytest_integration.log 2>&1 || { tail -30 $O/pytest_integration.log; exit 1; }
tail -2 $O/pytest_integration.log
bash tools/drain_sweep.sh $O/drain
H=tests/native/build/run_gpu_harness
for scene in wdas_cloud fire; do
  t=0; [ $scene = fire ] && t=1
  VPT_FEED_TRACE=1 timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/$scene.json out=$O/film.f32 w=1920 h=1080 \
    waves=256 grid_n=512 threads=1 batch=4096 temperature=$t > $O/trace_${scene}.log 2>&1
  echo "== $scene"; grep -v slotwait $O/trace_${scene}.log | tail -14
done
rm -f $O/film.f32
