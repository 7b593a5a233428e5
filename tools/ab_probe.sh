#!/bin/bash
# Timing-only A/B of probe builds (no parity: a probe changes the counters it feeds) against the
# default library: bench.py frames of each config, alternating default / each variant, <rounds> times.
#   bash tools/ab_probe.sh <tag> <configs> <rounds> lib1.so [lib2.so ...]
set -o pipefail
TAG=$1; CFGS=$2; ROUNDS=$3; shift 3
BASE=$PWD/volume_path_tracer_amd/lib/libvpt_amd.so
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for L in $BASE "$@"; do
    v=$(basename $L .so)
    for c in ${CFGS//,/ }; do
      f=$O/b_${v}_${c}_$r
      VPT_LIB=$PWD/${L#$PWD/} timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $f.json 2> $f.err || exit 1
      python -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$v $c $r', d['ms_per_step'], d['value'])"
    done
  done
done
