# final-kernel evidence: round profiles (PMC, rocprof, bench) then the other configs' bench lines
bash tools/profile_round.sh r01 || exit $?
bash tools/_gcmd_configs2.sh || exit $?
