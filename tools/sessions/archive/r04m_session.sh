set -u
# Final binary: every GPU test + smoke + the C1 / C2 / C4 / C3 bench lines (tools/final_check.sh).
bash tools/final_check.sh r04m || exit 1
