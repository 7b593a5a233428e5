#!/bin/bash
# r05ab6: 8 waves per SIMD for the density-only throughput kernel.  Experimental builds without the feed / pixel-mode
# item words in the lane's LDS state (19 words: 8 blocks per CU fit the LDS): w7n = that at 7 waves, w8 = at 8 waves
# (64 VGPRs); prev = HEAD.  One-launch C3 frames (tools/tune.py, best of 3), 3 rounds rotating.
set -u
O=gpurun_out/r05ab6; mkdir -p $O
L=$PWD/volume_path_tracer_amd/lib
one() {  # name lib config round
  VPT_LIB=$2 timeout -k 10 300 python tools/tune.py --config $3 --spp 256 --gates 6:8:36:4 --reps 3 > $O/$3_$1_$4.jsonl 2>&1 || exit 1
  echo "$3 round $4 $1 $(grep -o '"blocks": [0-9]*' $O/$3_$1_$4.jsonl) $(grep -o '"ms": [0-9.]*' $O/$3_$1_$4.jsonl)"
}
for r in 1 2 3; do
  case $r in 1) V="prev w7n w8";; 2) V="w8 prev w7n";; 3) V="w7n w8 prev";; esac
  for v in $V; do
    case $v in prev) lib=$L/libvpt_amd.so;; *) lib=$L/exp/libvpt_$v.so;; esac
    one $v $lib c3 $r
  done
done
echo "all steps done"
