#!/bin/bash
# r06r: every GPU test and smoke on the code after the run() setup work (split flatten / create, huge pages, kept
# host grids, repeated run() calls).
set -u
export TMPDIR=/tmp
STEPS="pytest smoke" bash tools/gpu_check.sh r06r || exit $?
grep -E "passed|failed" gpurun_out/r06r/pytest_gpu.log | tail -2
