#!/bin/bash
# The drop-in's drain (include/vpt_run.hpp: feeds) on the full C3 frame (1920x1080, 256 waves, 512^3 stand-in),
# one host thread, across feed windows and film periods; each line: the knobs and render_ms (bench.py's C3 frame
# is the one-launch reference).  The last run samples what main.cpp's window would show every 50 ms.
# Usage (GPU box): bash tools/drain_sweep.sh <out_dir> [extra harness args]
set -u
O=${1:-gpurun_out/drain}; shift || true
mkdir -p $O
H=tests/native/build/run_gpu_harness
run() {
  local tag=$1; shift
  timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/wdas_cloud.json out=$O/film_$tag.f32 w=1920 h=1080 waves=256 \
    grid_n=512 threads=1 batch=4096 "$@" > $O/$tag.log 2>&1 || { echo "$tag failed rc=$?"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $* $(grep render_ms $O/$tag.log)"
  rm -f $O/film_$tag.f32
}
run default "$@"
run pb0 push_batch=0 "$@"
run cost cost_order=1 "$@"
run nof_pb0 flush_ms=100000 push_batch=0 "$@"
run w18 window=262144 "$@"
run w20 window=1048576 "$@"
run f1000 flush_ms=1000 "$@"
run nof flush_ms=100000 "$@"
run default2 "$@"
run s50 sample_ms=50 "$@"
grep "^sample" $O/s50.log | head -40
# helper threads taking tokens for the driver (run()'s other worker threads), C3 and C4 (the token-bound one)
run h3 helpers=3 "$@"
timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/fire.json out=$O/film_c4.f32 w=1920 h=1080 waves=256 grid_n=512 \
  threads=1 batch=4096 temperature=1 > $O/c4_h0.log 2>&1 && echo "c4 helpers=0 $(grep render_ms $O/c4_h0.log)"
timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/fire.json out=$O/film_c4.f32 w=1920 h=1080 waves=256 grid_n=512 \
  threads=1 batch=4096 temperature=1 push_batch=0 > $O/c4_pb0.log 2>&1 && echo "c4 push_batch=0 $(grep render_ms $O/c4_pb0.log)"
timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/fire.json out=$O/film_c4.f32 w=1920 h=1080 waves=256 grid_n=512 \
  threads=1 batch=4096 temperature=1 helpers=3 > $O/c4_h3.log 2>&1 && echo "c4 helpers=3 $(grep render_ms $O/c4_h3.log)"
rm -f $O/film_c4.f32
