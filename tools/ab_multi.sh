#!/bin/bash
# Timing A/B of several variant library builds against the default one (no parity run: for builds whose samples
# cannot differ -- occupancy, unroll, gates): bench.py frames of each config, the builds in turn, <rounds> times.
#   bash tools/ab_multi.sh <tag> "<lib names ...>" [configs=c3,c4] [rounds=2]
set -o pipefail
TAG=$1; VARS=$2; CFGS=${3:-c3,c4}; ROUNDS=${4:-2}
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for c in ${CFGS//,/ }; do
    for v in base $VARS; do
      L=$PWD/volume_path_tracer_amd/lib/libvpt_amd.so; [ $v != base ] && L=$PWD/volume_path_tracer_amd/lib/libvpt_$v.so
      f=$O/b_${v}_${c}_$r
      VPT_LIB=$L timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $f.json 2> $f.err || exit 1
      python -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$v $c $r', d['ms_per_step'], d['value'])" | tee -a $O/summary.txt
    done
  done
done
