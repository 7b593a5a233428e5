#!/bin/bash
# r05c: feed traces of the drop-in's C3 and C4 frames (snapshot / final / clear timings), after the pusher's
# ring prefetch and the staged feeds' count skip.
set -eu
O=gpurun_out/r05c; mkdir -p $O
H=tests/native/build/run_gpu_harness
for scene in wdas_cloud fire; do
  t=0; [ $scene = fire ] && t=1
  for r in 1 2; do
    VPT_FEED_TRACE=1 timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/$scene.json out=$O/film.f32 w=1920 h=1080 \
      waves=256 grid_n=512 threads=1 batch=4096 temperature=$t > $O/trace_${scene}_$r.log 2>&1
    echo "== $scene $r"; grep -v slotwait $O/trace_${scene}_$r.log | tail -14
  done
  timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/$scene.json out=$O/film.f32 w=1920 h=1080 \
      waves=256 grid_n=512 threads=1 batch=4096 temperature=$t flush_ms=100000 > $O/nofilm_${scene}.log 2>&1
  echo "$scene nofilm $(grep render_ms $O/nofilm_${scene}.log)"
done
rm -f $O/film.f32
