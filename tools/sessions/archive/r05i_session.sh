#!/bin/bash
# r05i: the C3 8-GPU share's longest jobs alone (job log): a 32-wave frame, then its 24 longest
# jobs each in a launch of its own on the throughput and the latency kernel; C1's kernel counters (its bench line's request_frac / pipe_frac); then the drain sweep (C3 / C4 / C5
# drop-in frames, ADVICE r04: C5's snapshots).
set -u
O=gpurun_out/r05i; mkdir -p $O
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_joblog.so timeout -k 10 300 python tools/job_log.py --config c3 --spp 32 \
  --alone 24 --out $O/joblog32 > $O/joblog32.log 2>&1 || { tail $O/joblog32.log; exit 1; }
python -c "
import json; d = json.load(open('$O/joblog32/summary_c3.json'))
print({k: d[k] for k in ('span_ms', 'job_ms_max', 'work_over_lanes_ms', 'span_over_ideal')})
for r in d['longest_jobs']: print(r)"
bash tools/kernel_counters.sh r05 c1 > $O/counters_c1.txt 2>&1 || { tail $O/counters_c1.txt; exit 1; }
tail -6 $O/counters_c1.txt
bash tools/drain_sweep.sh $O/drain > $O/drain.txt 2>&1 || { tail $O/drain.txt; exit 1; }
cat $O/drain.txt | head -30
