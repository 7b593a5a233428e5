#!/bin/bash
# r05ab5: SGPR spills, continued.  prev = HEAD (launch arguments read where used); a = + the emission re-reads the
# scene at its own point (temperature kernel: 69 -> 6 v_readlane); b = a + the general HDDA step re-reads the
# density grid (walk loops: 0 v_readlane, +21..49 instructions for the loads).  Production parity tests with b,
# then one-launch C3 / C4 frames (tools/tune.py, best of 3), 3 rounds rotating.
set -u
O=gpurun_out/r05ab5; mkdir -p $O
L=$PWD/volume_path_tracer_amd/lib
VPT_LIB=$L/ab_b/libvpt_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_production.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
one() {  # name config round
  VPT_LIB=$L/ab_$1/libvpt_amd.so timeout -k 10 300 python tools/tune.py --config $2 --spp 256 --gates 6:8:36:4 --reps 3 > $O/$2_$1_$3.jsonl 2>&1 || exit 1
  echo "$2 round $3 $1 $(grep -o '"ms": [0-9.]*' $O/$2_$1_$3.jsonl)"
}
for r in 1 2 3; do
  case $r in 1) V="prev a b";; 2) V="b prev a";; 3) V="a b prev";; esac
  for c in c3 c4; do for v in $V; do one $v $c $r; done; done
done
echo "all steps done"
