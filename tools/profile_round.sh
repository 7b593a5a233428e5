#!/bin/bash
# Round evidence for profiles/: PMC passes over one C3 launch (fabric read requests by size, DRAM-bound
# requests, FETCH_SIZE / WRITE_SIZE, L2 hit/miss; one pass each, each under its own time limit),
# rocprofv3 --kernel-trace --stats of the bench, and the full bench.
# Usage (on the GPU box): bash tools/profile_round.sh <tag> [config]    e.g. r02 c3
# Only gpurun_out/ comes back: afterwards run tools/collect_profiles.sh <tag> here.
set -u
TAG=${1:-r02}; CFG=${2:-c3}; O=gpurun_out/${TAG}_${CFG}; mkdir -p $O profiles
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/$name.log; exit $rc; fi; }
i=0
while IFS= read -r P; do
  i=$((i+1))
  step pmc_$i 300 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$i -o run -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-dropin
done <<'PASSES'
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
PASSES
python3 tools/pmc_traffic.py ${TAG}_${CFG} $CFG $(python3 -c "from volume_path_tracer_amd.scenes import workload; print(workload('$CFG').spp)") $O/pmc_* || exit 1
cp profiles/${TAG}_${CFG}_pmc.json $O/
step rocprof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config $CFG --no-cpu-baseline --no-dropin
if [ "$CFG" = "c3" ]; then step bench 900 python3 bench.py; tail -1 $O/bench.log | cut -c1-400; fi
