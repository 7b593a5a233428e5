#!/bin/bash
# r06g: the kernels as committed (ordered film stored from the lane): film-order + production parity tests, then
# the roofline inputs refreshed on this binary: PMC traffic + kernel trace (C3, C4), kernel
# counter passes (C3, C4), strong-scaling emulation (C3 / C5 shares).
set -u
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_film_order.py tests/test_gpu_production.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/profile_round.sh r06g c3 || exit $?
bash tools/profile_round.sh r06g c4 || exit $?
bash tools/kernel_counters.sh r06g c3 || exit $?
bash tools/kernel_counters.sh r06g c4 || exit $?
bash tools/strong_emulation.sh r06g_strong || exit $?
