#!/bin/bash
# r05ab2: the feed protocol compiled into its own kernel instantiations (KernelEnvT<.., Feed>), so the one-launch
# kernels carry none of it (plain C3 kernel 5 143 -> 4 837 instructions, 120 -> 66 v_readlane).  The GPU suite,
# then one-launch C3 / C4 frames (tools/tune.py, best of 3) and drop-in frames (run_gpu_harness, 3 frames), the
# library before the urgent-fetch gate (prev) vs this one (new), 3 rounds alternating.
set -u
O=gpurun_out/r05ab2; mkdir -p $O
L=$PWD/volume_path_tracer_amd/lib
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
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
for r in 1 2 3; do
  if [ $((r % 2)) = 1 ]; then A=prev; B=new; else A=new; B=prev; fi
  for c in c3 c4; do
    for v in $A $B; do
      if [ $v = prev ]; then one prev $L/ab_prev/libvpt_amd.so $c $r; else one new $L/libvpt_amd.so $c $r; fi
    done
  done
  for sc in wdas_cloud fire; do
    for v in $A $B; do
      if [ $v = prev ]; then drop prev $L/ab_prev $sc $r; else drop new $L $sc $r; fi
    done
  done
done
echo "all steps done"
