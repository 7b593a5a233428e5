# final evidence for the committed tree: GPU tests + smoke, round profiles, other configs
bash tools/_gcmd_final.sh || exit $?
bash tools/profile_round.sh r01 || exit $?
bash tools/_gcmd_configs2.sh || exit $?
