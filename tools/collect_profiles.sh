#!/bin/bash
# Copy a profile_round.sh run (merged back under gpurun_out/<tag>) into the tracked profiles/.
set -e
TAG=${1:-r02}; CFG=${2:-c3}; O=gpurun_out/${TAG}_${CFG}
cp $O/${TAG}_${CFG}_pmc.json profiles/${TAG}_${CFG}_pmc.json
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) profiles/${TAG}_${CFG}_kernel_stats.csv
grep "\"metric\"" $O/rocprof.log | tail -1 > profiles/${TAG}_${CFG}_rocprof_bench.json
if [ -f $O/bench.log ]; then cp $O/bench.log profiles/${TAG}_${CFG}_bench.log; fi
ls -la profiles/
