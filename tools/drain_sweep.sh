#!/bin/bash
# The drop-in's drain (include/vpt_run.hpp: one staged feed, pusher and film threads) on the full C3 frame
# (1920x1080, 256 waves, 512^3 stand-in), the C4 frame and the C5 frame (3840x2160, 1 024 waves), one host thread, across the run-ahead bounds (hold /
# backlog), the cost tail and the film period; each line: the knobs and render_ms (bench.py's C3 frame is the
# one-launch reference), one warm-up frame and 3 timed frames per setting.  Then the provider alone (mode=tokens:
# the host-side floor) and a run sampling what main.cpp's window would show every 50 ms.
# Usage (GPU box): bash tools/drain_sweep.sh <out_dir> [extra harness args]
set -u
O=${1:-gpurun_out/drain}; shift || true
mkdir -p $O
H=tests/native/build/run_gpu_harness
run() {
  local tag=$1 scene=$2; shift 2
  local t=0; [ "$scene" = fire ] && t=1
  timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/$scene.json out=$O/film_$tag.f32 w=1920 h=1080 waves=256 \
    grid_n=512 threads=1 batch=4096 temperature=$t warmup=1 frames=3 "$@" > $O/$tag.log 2>&1 || { echo "$tag failed rc=$?"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $scene $* render_ms $(grep render_ms $O/$tag.log | awk '{print $3}' | tr '\n' ' ')"
  rm -f $O/film_$tag.f32
}
run c3_default wdas_cloud "$@"
run c3_nofilm wdas_cloud flush_ms=100000 "$@"
run c3_notail wdas_cloud cost_tail=0 "$@"
run c3_nochunks wdas_cloud cost_chunks=0 "$@"
run c3_hold2 wdas_cloud hold=917504 "$@"
run c3_hold6 wdas_cloud hold=2752512 "$@"
run c3_backlog_half wdas_cloud backlog=229376 "$@"
run c3_default2 wdas_cloud "$@"
run c4_default fire "$@"
run c4_nofilm fire flush_ms=100000 "$@"
run c4_default2 fire "$@"
# C5 (3840x2160, 1 024 waves): the 133-MB film's snapshots every 0.2 s (bench.py's C5 one-launch: ~5.2 s)
run c5_default wdas_cloud w=3840 h=2160 waves=1024 warmup=0 frames=2 "$@"
run c5_nofilm wdas_cloud w=3840 h=2160 waves=1024 warmup=0 frames=2 flush_ms=100000 "$@"
for th in 1 2; do
  timeout -k 10 60 $H config=volume_path_tracer_amd/scenes/wdas_cloud.json out=$O/x w=1920 h=1080 waves=256 mode=tokens \
    threads=$th > $O/tokens_$th.log 2>&1 && echo "provider alone: $(grep tokens_ms $O/tokens_$th.log)"
done
run c3_s50 wdas_cloud sample_ms=50 frames=1 warmup=0 "$@"
grep "^sample" $O/c3_s50.log | head -40
