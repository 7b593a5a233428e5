#!/bin/bash
# r05h: evidence passes: SQ / vector-memory counters of C2 without and with live-path
# compaction (period $1), the C3 8-GPU share's job log (32 waves, VPT_JOB_LOG build), and the PMC traffic passes
# plus kernel-trace summaries of C2 and C1 (tools/profile_round.sh) for their bench lines' roofline.traffic.
set -u
K=${1:-4}
O=gpurun_out/r05h; mkdir -p $O
bash tools/kernel_counters.sh r05 c2 > $O/counters_c2.txt 2>&1 || { tail $O/counters_c2.txt; exit 1; }
tail -12 $O/counters_c2.txt
bash tools/kernel_counters.sh r05cmp$K c2 --compaction $K > $O/counters_c2_cmp.txt 2>&1 || { tail $O/counters_c2_cmp.txt; exit 1; }
tail -12 $O/counters_c2_cmp.txt
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_joblog.so timeout -k 10 300 python tools/job_log.py --config c3 --spp 32 \
  --out $O/joblog32 > $O/joblog32.log 2>&1 || { tail $O/joblog32.log; exit 1; }
tail -c 1500 $O/joblog32.log
bash tools/profile_round.sh r05 c2 > $O/profile_c2.txt 2>&1 || { tail $O/profile_c2.txt; exit 1; }
bash tools/profile_round.sh r05 c1 > $O/profile_c1.txt 2>&1 || { tail $O/profile_c1.txt; exit 1; }
echo profiles done
