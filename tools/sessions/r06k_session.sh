#!/bin/bash
# r06k: the bench lines of every configuration on the round-6 code: C1 / C2 / C4 / C5 (with their CPU baselines,
# parity and drop-in records) and the default C3 line.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
for C in c1 c2 c4; do
  timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --cpu-budget 6 > $O/bench_$C.json 2> $O/bench_$C.err || exit 1
  cut -c1-200 $O/bench_$C.json
done
timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --cpu-budget 6 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
cut -c1-200 $O/bench_c5.json
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
cut -c1-200 $O/bench_c3.json
