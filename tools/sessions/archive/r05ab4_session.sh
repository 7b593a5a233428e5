#!/bin/bash
# r05ab4: as r05ab3, on the bench's own C2 / C1 paths (the latency kernel and its grid rule; tune.py's fixed grids
# run the throughput kernel): bench.py --config c2 / c1, 10 steps, no CPU baseline or drop-in, prev vs new, 3 rounds.
set -u
O=gpurun_out/r05ab4; mkdir -p $O
L=$PWD/volume_path_tracer_amd/lib
b() {  # name lib config round
  VPT_LIB=$2 timeout -k 10 300 python bench.py --config $3 --steps 10 --warmup 2 --no-cpu-baseline --no-dropin > $O/$3_$1_$4.log 2>&1 || { tail -5 $O/$3_$1_$4.log; exit 1; }
  echo "$3 round $4 $1 $(grep -o '"ms_per_step": [0-9.]*' $O/$3_$1_$4.log)"
}
for r in 1 2 3; do
  if [ $((r % 2)) = 1 ]; then A=prev; B=new; else A=new; B=prev; fi
  for c in c2 c1; do
    for v in $A $B; do
      if [ $v = prev ]; then b prev $L/ab_prev/libvpt_amd.so $c $r; else b new $L/libvpt_amd.so $c $r; fi
    done
  done
done
echo "all steps done"
