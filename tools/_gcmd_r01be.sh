# density evaluation inside the walk loop (VPT_EVAL_IN_WALK): parity, A/B C3 with gate_walk 4 / 8 / 16
export TMPDIR=/tmp; O=gpurun_out/r01be; mkdir -p $O
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_ew.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_ew.log 2>&1; rc=$?
echo "pytest ew rc=$rc"; tail -1 $O/pytest_ew.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/tune.py --spp 256 --gates 6:12:32:4 --reps 2 > $O/base.log 2>&1 || exit $?
echo "base $(grep Msps $O/base.log | tail -1 | cut -c100-200)"
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_ew.so timeout -k 10 300 python tools/tune.py --spp 256 --gates 6:12:32:4,6:12:32:8,6:12:32:16,6:12:24:8 --reps 2 > $O/ew.log 2>&1 || exit $?
grep Msps $O/ew.log | cut -c60-200
