#!/bin/bash
# Feed diagnostics on the full C3 frame: the drop-in's drain with VPT_FEED_TRACE=1 (feed opens / closes /
# slot waits / ends, ms) for no feed switch, a 16-wave frame and the full 256-wave frame.  Each run is capped
# at 75 s (a stalled feed ends by its lanes' 30 s deadline).  Usage (GPU box): bash tools/feed_diag.sh <out_dir>
set -u
O=${1:-gpurun_out/feed_diag}; mkdir -p $O
H=tests/native/build/run_gpu_harness
run() {
  local tag=$1; shift
  VPT_FEED_TRACE=1 timeout -k 10 75 $H config=volume_path_tracer_amd/scenes/wdas_cloud.json out=$O/film.f32 w=1920 h=1080 \
    grid_n=512 threads=1 batch=4096 "$@" > $O/$tag.log 2>&1
  local rc=$?
  echo "== $tag $* rc=$rc $(grep render_ms $O/$tag.log)"
  grep -c "^feed" $O/$tag.log
  grep -v "^feed" $O/$tag.log | tail -3
  grep "^feed" $O/$tag.log | head -12
  grep "^feed" $O/$tag.log | tail -8
  rm -f $O/film.f32
  [ $rc -eq 0 ] || [ $rc -eq 1 ]
}
run w16 waves=16 && run nof waves=256 flush_ms=100000 && run w256 waves=256 sample_ms=100
