#!/bin/bash
# Copy a profile_round.sh run (merged back under gpurun_out/<tag>) into the tracked profiles/.
set -e
TAG=${1:-r01}; O=gpurun_out/$TAG
cp $O/${TAG}_pmc.json profiles/${TAG}_pmc.json
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) profiles/${TAG}_c3_kernel_stats.csv
grep "\"metric\"" $O/rocprof.log | tail -1 > profiles/${TAG}_c3_rocprof_bench.json
cp $O/bench.log profiles/${TAG}_c3_bench.log
ls -la profiles/
