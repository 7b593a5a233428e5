#!/bin/bash
# A/B of the latency kernel (vpt_gpu_set_latency_kernel) on the latency-bound and partly filled workloads:
# C1, C2, and C3 shares of 16 / 32 waves (a GPU's share of the 1080p frame dealt over 16 / 8 GPUs), two
# alternating rounds; prints config, mode, ms_per_step.  Usage (GPU box): bash tools/lat_ab.sh <out_dir>
set -u
O=${1:-gpurun_out/lat_ab}; mkdir -p $O
one() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-dropin "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; j=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', j['config']['latency_kernel'], j['ms_per_step'], j['value'])"
}
for r in 1 2; do
  for m in off auto; do
    one c1_${m}_$r --config c1 --steps 10 --warmup 2 --latency-kernel $m
    one c2_${m}_$r --config c2 --steps 5 --warmup 1 --latency-kernel $m
    one c3s16_${m}_$r --config c3 --spp 16 --steps 5 --warmup 1 --latency-kernel $m
    one c3s32_${m}_$r --config c3 --spp 32 --steps 5 --warmup 1 --latency-kernel $m
  done
done
