#!/bin/bash
# r06i: occupancy and walk-unroll re-checks on the round-6 kernels: 6 waves per SIMD for the density kernel (w6),
# 5 / 7 for the temperature kernel (t5 / t7), walk-loop unroll 2 / 4 (u2 / u4; default 3).
set -u
export TMPDIR=/tmp
bash tools/ab_multi.sh r06i "w6 u2 u4" c3 2 || exit $?
bash tools/ab_multi.sh r06i_c4 "t5 t7 u2 u4" c4 2 || exit $?
