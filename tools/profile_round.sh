#!/bin/bash
# Round evidence for profiles/: full bench (with CPU baseline), rocprofv3 kernel-trace stats of the
# same bench, and the PMC traffic passes (FETCH_SIZE, WRITE_SIZE, TCC hit/miss), one pass each.
# Usage (on the GPU box): bash tools/profile_round.sh <tag>      e.g. r01
# Only gpurun_out/ comes back: afterwards run tools/collect_profiles.sh <tag> here.
set -u
TAG=${1:-r01}; O=gpurun_out/$TAG; mkdir -p $O profiles
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/$name.log; exit $rc; fi; }
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $P | cut -d' ' -f1)
  step pmc_$N 400 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$N -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
done
python3 tools/pmc_traffic.py ${TAG} c3 256 $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/pmc_TCC_HIT_sum || exit 1
cp profiles/${TAG}_pmc.json $O/
step rocprof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline

step bench 900 python3 bench.py
tail -1 $O/bench.log | cut -c1-400
