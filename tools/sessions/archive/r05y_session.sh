#!/bin/bash
# r05y: the drop-in after the progress() probe (kernel as before): integration GPU tests, then C3 / C4 / C2 / C1
# drop-in frames (1 warm-up + 3 each), two rounds.
set -u
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_integration.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
H=tests/native/build/run_gpu_harness
run() {
  local tag=$1 scene=$2; shift 2
  local t=0; [ "$scene" = fire ] && t=1
  VPT_DRAIN_TRACE=1 timeout -k 10 60 $H config=volume_path_tracer_amd/scenes/$scene.json out=$O/film.f32 threads=1 \
    batch=4096 temperature=$t warmup=1 frames=3 "$@" > $O/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc render_ms $(grep render_ms $O/$tag.log | awk '{print $3}' | tr '\n' ' ')"
  rm -f $O/film.f32
  [ $rc -eq 0 ] || exit $rc
}
for r in 1 2; do
  run c3_$r wdas_cloud w=1920 h=1080 waves=256 grid_n=512
  run c4_$r fire w=1920 h=1080 waves=256 grid_n=512
  run c2_$r wdas_cloud w=512 h=512 waves=64 grid_n=128 kind=0 dist=300
  run c1_$r wdas_cloud w=256 h=256 waves=4 grid_n=512
done
