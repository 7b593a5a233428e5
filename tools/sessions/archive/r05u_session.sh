#!/bin/bash
# r05u: round evidence for the headline configs on the round's final binary: PMC traffic passes + kernel-trace
# summary + bench for C3 (tools/profile_round.sh), the same for C4; then C3 / C4 kernel counters.
set -u
bash tools/profile_round.sh r05 c3 > gpurun_out/r05u_c3.txt 2>&1 || { tail gpurun_out/r05u_c3.txt; exit 1; }
tail -3 gpurun_out/r05u_c3.txt | cut -c1-300
bash tools/profile_round.sh r05 c4 > gpurun_out/r05u_c4.txt 2>&1 || { tail gpurun_out/r05u_c4.txt; exit 1; }
tail -3 gpurun_out/r05u_c4.txt | cut -c1-300
bash tools/kernel_counters.sh r05 c3 > gpurun_out/r05u_cnt_c3.txt 2>&1 || { tail gpurun_out/r05u_cnt_c3.txt; exit 1; }
bash tools/kernel_counters.sh r05 c4 > gpurun_out/r05u_cnt_c4.txt 2>&1 || { tail gpurun_out/r05u_cnt_c4.txt; exit 1; }
echo done
