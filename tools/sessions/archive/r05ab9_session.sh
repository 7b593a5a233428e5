#!/bin/bash
# r05ab9: the film commit after the fetch block (b: the job fetch's returning atomic no longer waits for the film
# adds; 1 VGPR more live, 4 scratch accesses) vs right after the finish block (prev = HEAD).  tools/tune.py C3 / C4,
# best of 3, 2 rounds alternating.
set -u
O=gpurun_out/r05ab9; mkdir -p $O
L=$PWD/volume_path_tracer_amd/lib
one() {  # name config round
  VPT_LIB=$L/ab_$1/libvpt_amd.so timeout -k 10 300 python tools/tune.py --config $2 --spp 256 --gates 6:8:36:4 --reps 3 > $O/$2_$1_$3.jsonl 2>&1 || exit 1
  echo "$2 round $3 $1 $(grep -o '"ms": [0-9.]*' $O/$2_$1_$3.jsonl)"
}
for r in 1 2; do
  if [ $r = 1 ]; then V="prev b"; else V="b prev"; fi
  for c in c3 c4; do for v in $V; do one $v $c $r; done; done
done
echo "all steps done"
