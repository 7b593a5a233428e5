#!/bin/bash
# r06zb: A/B of two cheap walk-loop variants against the default build (timing only; results cannot differ:
# the same instructions' values): the walk index as two full-rate v_mad_u32_u24 (libvpt_mad24.so), and C3 on the
# run-skipping kernel variant (libvpt_runs0.so, VPT_RUNS_MIN_FRACTION 0).  Then the mad24 build's production
# parity tests.
set -u
export TMPDIR=/tmp
bash tools/ab_multi.sh r06zb "mad24 runs0" c3,c4 2 || exit $?
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_mad24.so timeout -k 10 400 python -u -m pytest tests/test_gpu_production.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r06zb/pytest_mad24.log 2>&1 || { tail -20 gpurun_out/r06zb/pytest_mad24.log; exit 1; }
tail -1 gpurun_out/r06zb/pytest_mad24.log
