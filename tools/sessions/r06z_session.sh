#!/bin/bash
# r06z: the roofline inputs refreshed on the final binary (its kernel arguments grew by the ordered drop-in frame's
# fields, so the code objects differ from r06g's): PMC traffic + kernel trace (C3, C4), kernel counter passes.
set -u
export TMPDIR=/tmp
bash tools/profile_round.sh r06z c3 || exit $?
bash tools/profile_round.sh r06z c4 || exit $?
bash tools/kernel_counters.sh r06z c3 || exit $?
bash tools/kernel_counters.sh r06z c4 || exit $?
