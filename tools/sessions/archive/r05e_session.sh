#!/bin/bash
# r05e: the whole GPU suite and smoke on the r05 drop-in + kernel, then bench.py C3 (with its new dropin record) and C4.
set -u
STEPS="pytest smoke bench" bash tools/gpu_check.sh r05e || exit 1
timeout -k 10 600 python bench.py --config c4 --no-cpu-baseline > gpurun_out/r05e/bench_c4.log 2>&1; tail -1 gpurun_out/r05e/bench_c4.log
