#!/bin/bash
# r06e: roofline inputs refreshed on the current binaries: PMC traffic passes + kernel trace for
# C3 and C4 (tools/profile_round.sh), kernel counter passes for C3 and C4 (tools/kernel_counters.sh), and the
# strong-scaling emulation (tools/strong_emulation.sh: C3 and C5 shares on one GPU).
set -u
export TMPDIR=/tmp
bash tools/profile_round.sh r06e c3 || exit $?
bash tools/profile_round.sh r06e c4 || exit $?
bash tools/kernel_counters.sh r06e c3 || exit $?
bash tools/kernel_counters.sh r06e c4 || exit $?
bash tools/strong_emulation.sh r06e_strong || exit $?
