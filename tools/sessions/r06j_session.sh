#!/bin/bash
# r06j: every GPU test and smoke on the round-6 code (the round-end GPU tier, rehearsed).
set -u
export TMPDIR=/tmp
STEPS="pytest smoke" bash tools/gpu_check.sh r06j || exit $?
grep -E "passed|failed" gpurun_out/r06j/pytest_gpu.log | tail -2
