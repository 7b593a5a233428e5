set -u
# Round-end evidence, part 1: every GPU test + smoke + C1 / C2 / C4 / C3 bench lines (final_check.sh), then the
# drop-in's drain sweep (feeds, cost batches, progressive film; tools/drain_sweep.sh).
bash tools/final_check.sh r04z || exit 1
bash tools/drain_sweep.sh gpurun_out/r04z/drain || exit 1
