#!/bin/bash
# r05ab8: film adds regrouped per finish pass (lane 3k + c adds component c of the pass's k-th sample: one memory-side
# atomic request per sample instead of three) vs HEAD (prev).  Production / integration / parity GPU tests, then
# one-launch C3 / C4 frames (tools/tune.py, best of 3) and drop-in frames, 2 rounds alternating.
set -u
O=gpurun_out/r05ab8; mkdir -p $O
L=$PWD/volume_path_tracer_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_integration.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
one() {  # name lib config round
  VPT_LIB=$2 timeout -k 10 300 python tools/tune.py --config $3 --spp 256 --gates 6:8:36:4 --reps 3 > $O/$3_$1_$4.jsonl 2>&1 || exit 1
  echo "$3 round $4 $1 $(grep -o '"ms": [0-9.]*' $O/$3_$1_$4.jsonl)"
}
drop() {  # name libdir scene round
  local t=0; [ "$3" = fire ] && t=1
  LD_LIBRARY_PATH=$2${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 60 tests/native/build/run_gpu_harness \
    config=volume_path_tracer_amd/scenes/$3.json out=$O/film.f32 w=1920 h=1080 waves=256 grid_n=512 threads=1 batch=4096 \
    temperature=$t warmup=1 frames=3 > $O/drop_$3_$1_$4.log 2>&1 || exit 1
  echo "drop $3 round $4 $1 render_ms $(grep render_ms $O/drop_$3_$1_$4.log | awk '{print $3}' | tr '\n' ' ')"
  rm -f $O/film.f32
}
for r in 1 2; do
  if [ $r = 1 ]; then V="prev new"; else V="new prev"; fi
  for c in c3 c4; do for v in $V; do
    if [ $v = prev ]; then one prev $L/ab_prev/libvpt_amd.so $c $r; else one new $L/libvpt_amd.so $c $r; fi
  done; done
  for sc in wdas_cloud fire; do for v in $V; do
    if [ $v = prev ]; then drop prev $L/ab_prev $sc $r; else drop new $L $sc $r; fi
  done; done
done
echo "all steps done"
