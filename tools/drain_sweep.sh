#!/bin/bash
# The drop-in's drain (include/vpt_run.hpp) on the full C3 frame (1920x1080, 256 waves, 512^3 stand-in),
# one host thread, across round sizes / rounds in flight / grid policy; each line: the knobs and render_ms.
# Usage (GPU box): bash tools/drain_sweep.sh <out_dir> [extra harness args]
set -u
O=${1:-gpurun_out/drain}; shift || true
mkdir -p $O
H=tests/native/build/run_gpu_harness
T=32400
run() {
  local tag=$1; shift
  timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/wdas_cloud.json out=$O/film_$tag.f32 w=1920 h=1080 waves=256 \
    grid_n=512 threads=1 "$@" > $O/$tag.log 2>&1 || { echo "$tag failed rc=$?"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $* $(grep render_ms $O/$tag.log)"
  rm -f $O/film_$tag.f32
}
run one_launch batch=$((256*T)) rounds=1 "$@"
run b8_r1 batch=$((8*T)) rounds=1 "$@"
run b8_r2 batch=$((8*T)) rounds=2 "$@"
run b8_r3 batch=$((8*T)) rounds=3 "$@"
run b16_r2 batch=$((16*T)) rounds=2 "$@"
run b32_r2 batch=$((32*T)) rounds=2 "$@"
run b8_r2_full batch=$((8*T)) rounds=2 grid_blocks=1792 "$@"
run b16_r2_full batch=$((16*T)) rounds=2 grid_blocks=1792 "$@"
run b8_r2_s50 batch=$((8*T)) rounds=2 sample_ms=50 "$@"
grep "^sample" $O/b8_r2_s50.log | head -40
