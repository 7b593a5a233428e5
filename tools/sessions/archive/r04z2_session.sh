set -u
# Round-end evidence, part 2: the C3 and C4 profiles (PMC traffic passes, rocprofv3 --kernel-trace --stats of
# the bench, the full C3 bench) and the C3 kernel counters.  Copy into profiles/ with tools/collect_profiles.sh.
bash tools/profile_round.sh r04 c3 || exit 1
bash tools/profile_round.sh r04 c4 || exit 1
bash tools/kernel_counters.sh r04 c3 || exit 1
