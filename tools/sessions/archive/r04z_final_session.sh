set -u
# Round-end evidence on the final binary: every GPU test + smoke + C1/C2/C4/C3 bench lines (final_check.sh),
# then the C3 and C4 profiles (PMC traffic passes, rocprofv3 --kernel-trace --stats of the bench, the full C3
# bench) and the C3 kernel counters.  Copy into profiles/ afterwards with tools/collect_profiles.sh r04 c3|c4.
bash tools/final_check.sh r04z || exit 1
bash tools/profile_round.sh r04 c3 || exit 1
bash tools/profile_round.sh r04 c4 || exit 1
bash tools/kernel_counters.sh r04 c3 || exit 1
