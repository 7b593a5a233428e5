#!/bin/bash
# Strong scaling on one GPU: the per-rank share of a frame dealt over N ranks is a bench run with
# spp/N waves (waves 1..spp/N; every wave costs about the same), so t(spp) / t(spp/N) bounds the N-GPU
# speedup from above (it leaves out the film all-reduce, ~1 ms on xGMI, and any inter-GPU effect).
# Usage (GPU box): bash tools/strong_emulation.sh <tag>   -> gpurun_out/<tag>/strong_*.json
set -u
O=gpurun_out/${1:-strong}; mkdir -p $O; export TMPDIR=/tmp
for spec in "c3 256" "c3 128" "c3 64" "c3 32" "c5 1024" "c5 256" "c5 128"; do
  set -- $spec
  timeout -k 10 300 python3 bench.py --config $1 --spp $2 --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/strong_$1_$2.json 2> $O/strong_$1_$2.err
  rc=$?; echo "$1 spp $2 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/strong_$1_$2.json)"; if [ $rc -ne 0 ]; then tail -3 $O/strong_$1_$2.err; exit $rc; fi
done
