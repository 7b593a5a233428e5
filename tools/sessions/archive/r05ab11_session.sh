#!/bin/bash
# r05ab11: the temperature kernel at 5 waves per SIMD (t5: 85 VGPRs, no scratch) vs 6 (HEAD: 80 VGPRs, 12 B of
# scratch reloaded in the emission) after the film regroup.  tools/tune.py C4, best of 3, 3 rounds alternating.
set -u
O=gpurun_out/r05ab11; mkdir -p $O
L=$PWD/volume_path_tracer_amd/lib
one() {  # name lib round
  VPT_LIB=$2 timeout -k 10 300 python tools/tune.py --config c4 --spp 256 --gates 6:8:36:4 --reps 3 > $O/c4_$1_$3.jsonl 2>&1 || exit 1
  echo "c4 round $3 $1 $(grep -o '"blocks": [0-9]*' $O/c4_$1_$3.jsonl) $(grep -o '"ms": [0-9.]*' $O/c4_$1_$3.jsonl)"
}
for r in 1 2 3; do
  if [ $((r % 2)) = 1 ]; then V="prev t5"; else V="t5 prev"; fi
  for v in $V; do
    if [ $v = prev ]; then one prev $L/libvpt_amd.so $r; else one t5 $L/exp/libvpt_t5.so $r; fi
  done
done
echo "all steps done"
