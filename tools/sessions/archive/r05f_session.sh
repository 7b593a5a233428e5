#!/bin/bash
# r05f: C4 drop-in frame-to-frame variance: 6 frames with feed traces; the provider alone 3 times.
set -u
O=gpurun_out/r05f; mkdir -p $O
H=tests/native/build/run_gpu_harness
VPT_FEED_TRACE=1 VPT_DRAIN_TRACE=1 timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/fire.json out=$O/film.f32 w=1920 h=1080 \
  waves=256 grid_n=512 threads=1 batch=4096 temperature=1 frames=6 > $O/trace_c4.log 2>&1
grep -E "open_stg|launch|close|ended|cleared|render_ms|drain" $O/trace_c4.log
for i in 1 2 3; do timeout -k 10 60 $H config=volume_path_tracer_amd/scenes/fire.json out=$O/x w=1920 h=1080 waves=256 mode=tokens threads=1 | grep tokens_ms; done
VPT_FEED_TRACE=1 VPT_DRAIN_TRACE=1 timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/fire.json out=$O/film.f32 w=1920 h=1080 \
  waves=256 grid_n=512 threads=1 batch=4096 temperature=1 frames=6 flush_ms=100000 > $O/trace_c4_nofilm.log 2>&1
grep -E "render_ms|drain" $O/trace_c4_nofilm.log
rm -f $O/film.f32 $O/x
# C2's SIMT census on the latency kernel with the context's gates (its production launch): live lanes per wave
# iteration (PB_ITER), lanes per state at walk-loop iterations -- the premise of live-path compaction
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_prof.so timeout -k 10 300 python tools/tune.py --config c2 --spp 64 \
  --gates 6:8:36:4 --blocks 512 --lat-kernel 1 --lat-ungated 0 --profile --reps 1 > $O/c2_profile.jsonl 2>$O/c2_profile.err
cat $O/c2_profile.jsonl
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_analytic_multiscatter.py \
  > $O/pytest_multiscatter.log 2>&1; grep -E "PASSED|FAILED|passed|failed|variant|{" $O/pytest_multiscatter.log | tail -12
