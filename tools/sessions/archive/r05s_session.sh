#!/bin/bash
# r05s: the ring's backlog target now that its estimate is right (16 hint slots, the waiting word): C3 / C4 drop-in
# frames with backlog = the lanes (default) / half / a quarter, and the r05 library before the fix (prev) as the
# reference; alternating, 3 rounds, 1 warm-up + 3 frames each.
set -u
O=gpurun_out/r05s; mkdir -p $O
H=tests/native/build/run_gpu_harness
run() {
  local tag=$1 lib=$2 scene=$3; shift 3
  local t=0; [ "$scene" = fire ] && t=1
  local lp=""; [ "$lib" = prev ] && lp=$PWD/volume_path_tracer_amd/lib/ab_prev
  LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} VPT_DRAIN_TRACE=1 timeout -k 10 30 $H \
    config=volume_path_tracer_amd/scenes/$scene.json out=$O/film.f32 w=1920 h=1080 waves=256 grid_n=512 threads=1 \
    batch=4096 temperature=$t warmup=1 frames=3 "$@" > $O/$tag.log 2>&1
  local rc=$?
  echo "$tag $* rc=$rc render_ms $(grep render_ms $O/$tag.log | awk '{print $3}' | tr '\n' ' ')"
  rm -f $O/film.f32
  [ $rc -eq 0 ] || exit $rc
}
for r in 1 2 3; do
  run c3_prev_$r prev wdas_cloud
  run c3_b1_$r new wdas_cloud
  run c3_b2_$r new wdas_cloud backlog=229376
  run c3_b4_$r new wdas_cloud backlog=114688
  run c4_prev_$r prev fire
  run c4_b1_$r new fire
  run c4_b2_$r new fire backlog=196608
  run c4_b4_$r new fire backlog=98304
done
