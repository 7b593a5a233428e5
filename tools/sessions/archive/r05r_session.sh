#!/bin/bash
# r05r: A/B on one box -- the drop-in's C4 / C3 frames with the library before (prev: one backlog-hint word) and
# after (new: 16 hint slots + the 2-ms staleness rule), alternating, 4 rounds; the harness is the same binary.
set -u
O=gpurun_out/r05r; mkdir -p $O
H=tests/native/build/run_gpu_harness
run() {
  local tag=$1 lib=$2 scene=$3; shift 3
  local t=0; [ "$scene" = fire ] && t=1
  local lp=""; [ "$lib" = prev ] && lp=$PWD/volume_path_tracer_amd/lib/ab_prev
  LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} VPT_FEED_TRACE=1 VPT_DRAIN_TRACE=1 timeout -k 10 30 $H \
    config=volume_path_tracer_amd/scenes/$scene.json out=$O/film.f32 w=1920 h=1080 waves=256 grid_n=512 threads=1 \
    batch=4096 temperature=$t warmup=1 frames=3 "$@" > $O/$tag.log 2>&1
  local rc=$?
  echo "$tag $* rc=$rc render_ms $(grep render_ms $O/$tag.log | awk '{print $3}' | tr '\n' ' ') blocked $(grep taker_blocked $O/$tag.log | awk '{print $5}' | tr '\n' ' ') stale $(grep -c ' stale ' $O/$tag.log)"
  rm -f $O/film.f32
  [ $rc -eq 0 ] || exit $rc
}
for r in 1 2 3 4; do
  run c4_prev_$r prev fire
  run c4_new_$r new fire
  run c3_prev_$r prev wdas_cloud
  run c3_new_$r new wdas_cloud
done
