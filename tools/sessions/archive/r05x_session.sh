#!/bin/bash
# r05x: the feed's wavefront reservations (never past the published count) and the early launch (after the first
# pushed chunk; drain asks progress() after 64 K tokens): the whole GPU suite, then drop-in frames of the
# library + harness before (prev) and after (new), C3 / C4 alternating, 3 rounds; C1 / C2 drop-in once.
set -u
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
run() {
  local tag=$1 ver=$2 scene=$3; shift 3
  local t=0; [ "$scene" = fire ] && t=1
  local H=tests/native/build/run_gpu_harness lp=""
  [ "$ver" = prev ] && H=tests/native/build/run_gpu_harness_prev && lp=$PWD/volume_path_tracer_amd/lib/ab_prev
  LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} VPT_FEED_TRACE=1 VPT_DRAIN_TRACE=1 timeout -k 10 60 $H \
    config=volume_path_tracer_amd/scenes/$scene.json out=$O/film.f32 grid_n=512 threads=1 batch=4096 temperature=$t \
    warmup=1 frames=3 "$@" > $O/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc render_ms $(grep render_ms $O/$tag.log | awk '{print $3}' | tr '\n' ' ') slotwaits $(grep -c slotwait $O/$tag.log) launch_ms $(grep ' launch ' $O/$tag.log | head -2 | awk '{print $2}' | tr '\n' ' ')"
  rm -f $O/film.f32
  [ $rc -eq 0 ] || exit $rc
}
for r in 1 2 3; do
  run c3_prev_$r prev wdas_cloud w=1920 h=1080 waves=256
  run c3_new_$r new wdas_cloud w=1920 h=1080 waves=256
  run c4_prev_$r prev fire w=1920 h=1080 waves=256
  run c4_new_$r new fire w=1920 h=1080 waves=256
done
run c1_new new wdas_cloud w=256 h=256 waves=4
run c4b4_new new fire w=1920 h=1080 waves=256 backlog=98304
