#!/bin/bash
# r05ab10: what the latency kernel's per-lane film adds cost on the bench's C2 / C1 paths: a timing build without
# them (nofilmlat; the LDS-state kernels unchanged) vs HEAD.  bench.py 10 steps, 2 rounds alternating.
set -u
O=gpurun_out/r05ab10; mkdir -p $O
L=$PWD/volume_path_tracer_amd/lib
b() {  # name lib config round
  VPT_LIB=$2 timeout -k 10 300 python bench.py --config $3 --steps 10 --warmup 2 --no-cpu-baseline --no-dropin > $O/$3_$1_$4.log 2>&1 || { tail -5 $O/$3_$1_$4.log; exit 1; }
  echo "$3 round $4 $1 $(grep -o '"ms_per_step": [0-9.]*' $O/$3_$1_$4.log)"
}
for r in 1 2; do
  if [ $r = 1 ]; then V="prev nofilmlat"; else V="nofilmlat prev"; fi
  for c in c2 c1; do for v in $V; do
    if [ $v = prev ]; then b prev $L/libvpt_amd.so $c $r; else b $v $L/exp/libvpt_$v.so $c $r; fi
  done; done
done
echo "all steps done"
