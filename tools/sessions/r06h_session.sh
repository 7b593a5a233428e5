#!/bin/bash
# r06h: a whole-suite checkpoint on the round-6 code: every GPU test, smoke, then the bench lines of C1 / C2 / C4 /
# C5 and the default C3 (tools/final_check.sh, plus C5).
set -u
export TMPDIR=/tmp
bash tools/final_check.sh r06h || exit $?
O=gpurun_out/r06h
timeout -k 10 600 python bench.py --config c5 --steps 2 --warmup 1 --cpu-budget 6 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
cut -c1-300 $O/bench_c5.json
