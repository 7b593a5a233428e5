#!/bin/bash
# r05ab7: what the per-sample film atomics cost now: an experimental build whose film_add issues no atomics (nofilm)
# vs HEAD (prev).  One-launch C3 / C4 frames (tools/tune.py, best of 3), 2 rounds alternating.  Then C5 on HEAD.
set -u
O=gpurun_out/r05ab7; mkdir -p $O
L=$PWD/volume_path_tracer_amd/lib
one() {  # name lib config round
  VPT_LIB=$2 timeout -k 10 300 python tools/tune.py --config $3 --spp 256 --gates 6:8:36:4 --reps 3 > $O/$3_$1_$4.jsonl 2>&1 || exit 1
  echo "$3 round $4 $1 $(grep -o '"ms": [0-9.]*' $O/$3_$1_$4.jsonl)"
}
for r in 1 2; do
  if [ $r = 1 ]; then V="prev nofilm"; else V="nofilm prev"; fi
  for c in c3 c4; do for v in $V; do
    case $v in prev) lib=$L/libvpt_amd.so;; *) lib=$L/exp/libvpt_$v.so;; esac
    one $v $lib $c $r
  done; done
done
timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
grep '^{"metric"' $O/bench_c5.log | tail -1 | cut -c1-250
echo "all steps done"
