#!/bin/bash
# r05t (second run: 4 hint slots in the word's line, the ring back at word 8): which part of the backlog-hint fix slows some drop-in frames: 16 hint slots vs one word (VPT_HINT_SLOTS=1),
# the waiting word on / off (VPT_FEED_WAITING=0), against the library before the fix (prev); C4 and C3, 3 rounds.
set -u
O=gpurun_out/r05t; mkdir -p $O
H=tests/native/build/run_gpu_harness
run() {
  local tag=$1 lib=$2 scene=$3 slots=$4 waitw=$5
  local t=0; [ "$scene" = fire ] && t=1
  local lp=""; [ "$lib" = prev ] && lp=$PWD/volume_path_tracer_amd/lib/ab_prev
  LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} VPT_HINT_SLOTS=$slots VPT_FEED_WAITING=$waitw VPT_DRAIN_TRACE=1 \
    timeout -k 10 30 $H config=volume_path_tracer_amd/scenes/$scene.json out=$O/film.f32 w=1920 h=1080 waves=256 grid_n=512 \
    threads=1 batch=4096 temperature=$t warmup=1 frames=3 > $O/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc render_ms $(grep render_ms $O/$tag.log | awk '{print $3}' | tr '\n' ' ') blocked $(grep taker_blocked $O/$tag.log | awk '{print $5}' | tr '\n' ' ')"
  rm -f $O/film.f32
  [ $rc -eq 0 ] || exit $rc
}
for r in 1 2 3; do
  for sc in fire wdas_cloud; do
    run ${sc}_s4w1_$r new $sc 4 1
    run ${sc}_prev_$r prev $sc 4 1
    run ${sc}_s1w0_$r new $sc 1 0
    run ${sc}_s1w1_$r new $sc 1 1
  done
done
