#!/bin/bash
# C2 and C3 32-wave shares: throughput kernel vs the latency kernel forced with its own (ungated) gates vs forced
# with the context's gates, three alternating rounds.  Usage (GPU box): bash tools/lat_gated_ab.sh <out_dir>
set -u
O=${1:-gpurun_out/lat_gated}; mkdir -p $O
one() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-dropin "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json; j=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', j['config']['latency_kernel'], j['ms_per_step'], j['value'])"
}
for r in 1 2 3; do
  for m in off on gated; do
    one c2_${m}_$r --config c2 --steps 5 --warmup 1 --latency-kernel $m
    one c3s32_${m}_$r --config c3 --spp 32 --steps 5 --warmup 1 --latency-kernel $m
  done
done
