#!/bin/bash
# r05u2: the urgent-fetch gate (a feed lane holding an unread item runs its wavefront's fetch block at once), then
# launching the feed earlier (VPT_FEED_LAUNCH_DIV 4 / 16) -- against the library + harness before (prev);
# C3 / C4 drop-in frames with feed traces, 3 rounds; the feed tests first.
set -u
O=gpurun_out/r05u2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_integration.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {
  local tag=$1 ver=$2 div=$3 scene=$4
  local t=0; [ "$scene" = fire ] && t=1
  local H=tests/native/build/run_gpu_harness lp=""
  [ "$ver" = prev ] && H=tests/native/build/run_gpu_harness_prev && lp=$PWD/volume_path_tracer_amd/lib/ab_prev
  LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} VPT_FEED_LAUNCH_DIV=$div VPT_FEED_TRACE=1 timeout -k 10 60 $H \
    config=volume_path_tracer_amd/scenes/$scene.json out=$O/film.f32 w=1920 h=1080 waves=256 grid_n=512 threads=1 batch=4096 \
    temperature=$t warmup=1 frames=3 > $O/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc render_ms $(grep render_ms $O/$tag.log | awk '{print $3}' | tr '\n' ' ') slotwaits $(grep -c slotwait $O/$tag.log)"
  rm -f $O/film.f32
  [ $rc -eq 0 ] || exit $rc
}
for r in 1 2 3; do
  run c3_prev_$r prev 1 wdas_cloud
  run c3_new1_$r new 1 wdas_cloud
  run c3_new4_$r new 4 wdas_cloud
  run c3_new16_$r new 16 wdas_cloud
  run c4_prev_$r prev 1 fire
  run c4_new1_$r new 1 fire
  run c4_new4_$r new 4 fire
  run c4_new16_$r new 16 fire
done
