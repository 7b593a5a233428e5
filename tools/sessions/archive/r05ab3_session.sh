#!/bin/bash
# r05ab3: the kernels read their launch arguments through an opaque pointer to the argument segment (KernelArgs,
# scalar loads where used) instead of keeping them live in SGPRs: SGPR spill reloads outside the walk loops
# 120 -> 14 (plain), 104 -> 4 (run-skipping, but 18 inside its walk loop), 100 -> 69 (temperature).  The parity
# and feed tests, then one-launch frames of C3 / C4 / C2 / C1 (tools/tune.py, best of 3), HEAD before (prev) vs this
# one (new), 3 rounds alternating.
set -u
O=gpurun_out/r05ab3; mkdir -p $O
L=$PWD/volume_path_tracer_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_integration.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
one() {  # name lib config spp round
  VPT_LIB=$2 timeout -k 10 300 python tools/tune.py --config $3 --spp $4 --gates 6:8:36:4 --reps 3 > $O/$3_$1_$5.jsonl 2>&1 || exit 1
  echo "$3 round $5 $1 $(grep -o '"ms": [0-9.]*' $O/$3_$1_$5.jsonl)"
}
for r in 1 2 3; do
  if [ $((r % 2)) = 1 ]; then A=prev; B=new; else A=new; B=prev; fi
  for cs in c3:256 c4:256 c2:64 c1:4; do
    for v in $A $B; do
      if [ $v = prev ]; then one prev $L/ab_prev/libvpt_amd.so ${cs%%:*} ${cs##*:} $r; else one new $L/libvpt_amd.so ${cs%%:*} ${cs##*:} $r; fi
    done
  done
done
echo "all steps done"
