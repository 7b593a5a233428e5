#!/bin/bash
# r05n: the drop-in with its pusher / film threads bound to the GPU's NUMA node (vpt_gpu_bind_thread_near):
# the taker (the calling thread) left to the OS, on node 0 or on node 1; C4 and C3, 1 warm-up + 3 frames, 3 rounds.
set -u
O=gpurun_out/r05n; mkdir -p $O
H=tests/native/build/run_gpu_harness
run() {
  local tag=$1 scene=$2; shift 2
  local t=0; [ "$scene" = fire ] && t=1
  VPT_DRAIN_TRACE=1 timeout -k 10 60 $H config=volume_path_tracer_amd/scenes/$scene.json out=$O/film.f32 w=1920 h=1080 \
    waves=256 grid_n=512 threads=1 batch=4096 temperature=$t warmup=1 frames=3 "$@" > $O/$tag.log 2>&1
  local rc=$?
  echo "$tag $* rc=$rc render_ms $(grep render_ms $O/$tag.log | awk '{print $3}' | tr '\n' ' ') blocked $(grep taker_blocked $O/$tag.log | awk '{print $5}' | tr '\n' ' ')"
  rm -f $O/film.f32
  [ $rc -eq 0 ] || exit $rc
}
for r in 1 2 3; do
  run c4_os_$r fire
  run c4_n0_$r fire taker_node=0
  run c4_n1_$r fire taker_node=1
  run c3_os_$r wdas_cloud
  run c3_n1_$r wdas_cloud taker_node=1
done
