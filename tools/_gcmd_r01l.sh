export TMPDIR=/tmp; O=gpurun_out/r01l; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 $O/pytest.log
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd.so timeout -k 10 300 python tools/tune.py --spp 32 --gates 8:8:16:0,8:8:16:8,8:8:16:16,8:8:16:24,8:8:16:32,8:8:16:48 --reps 2 > $O/tune_def.log 2>&1 || exit $?
grep Msps $O/tune_def.log
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_nolook.so timeout -k 10 300 python tools/tune.py --spp 32 --gates 8:8:16:0,8:8:16:16 --reps 2 > $O/tune_nolook.log 2>&1 || exit $?
grep Msps $O/tune_nolook.log
