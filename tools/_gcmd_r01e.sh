export TMPDIR=/tmp; O=gpurun_out/r01e; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 $O/pytest.log
timeout -k 10 500 python tools/tune.py --spp 32 --gates 1:1:1,8:8:1,8:8:8,8:8:16,16:16:16,8:16:24,16:8:16 --reps 1 > $O/tune.log 2>&1 || exit $?
grep Msps $O/tune.log
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_prof.so timeout -k 10 300 python tools/tune.py --spp 32 --gates 8:8:1,8:8:16 --reps 1 --profile > $O/prof.log 2>&1 || exit $?
grep profile $O/prof.log
