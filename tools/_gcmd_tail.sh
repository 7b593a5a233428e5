#!/bin/bash
# VPT_ORDER_COST_TAIL sweep of the tile-major tail length on the full C3 frame.
export TMPDIR=/tmp; O=gpurun_out/tail2; mkdir -p $O
for S in ${SPPS:-32 256 512}; do for TL in ${TAILS:-0 40 80 160}; do
  timeout -k 10 300 python tools/tune.py --spp $S --gates 8:12:24:4 --reps 2 --order 3 --tail $TL > $O/s$S.t$TL.log 2>&1 || exit $?
  echo "spp=$S tail=$TL $(grep Msps $O/s$S.t$TL.log | tail -1 | cut -c1-200)"
done; done
