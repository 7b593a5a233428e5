#!/bin/bash
# r05end2 (a): the round's closing evidence for C3 on the final kernels: PMC traffic passes, rocprofv3 kernel trace of
# the bench, the full bench line (tools/profile_round.sh).
set -u
# (r05end2: the same after the film regroup)
bash tools/profile_round.sh r05end2 c3
