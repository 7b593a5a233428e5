#!/bin/bash
# r05k: the drop-in's start and tail -- launching the feed at 1/4 or 1/16 of the lanes (VPT_FEED_LAUNCH_DIV),
# and for C4 smaller run-ahead bounds (backlog / hold); 1 warm-up + 3 frames each, alternating.
set -u
O=gpurun_out/r05k; mkdir -p $O
H=tests/native/build/run_gpu_harness
run() {
  local tag=$1 scene=$2 div=$3; shift 3
  local t=0; [ "$scene" = fire ] && t=1
  VPT_FEED_LAUNCH_DIV=$div timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/$scene.json out=$O/film.f32 w=1920 h=1080 \
    waves=256 grid_n=512 threads=1 batch=4096 temperature=$t warmup=1 frames=3 "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag div=$div $* render_ms $(grep render_ms $O/$tag.log | awk '{print $3}' | tr '\n' ' ')"
  rm -f $O/film.f32
}
for r in 1 2; do
  run c3_div1_$r wdas_cloud 1
  run c3_div4_$r wdas_cloud 4
  run c3_div16_$r wdas_cloud 16
  run c4_div1_$r fire 1
  run c4_div4_$r fire 4
  run c4_div16_$r fire 16
  run c4_b4_$r fire 1 backlog=98304
  run c4_b4h1_$r fire 1 backlog=98304 hold=393216
done
