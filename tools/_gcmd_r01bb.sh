# LaneCold 19 words (terminated as a state, stencil refreshes tallied): 8 waves/SIMD probe
export TMPDIR=/tmp; O=gpurun_out/r01bb; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_w8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_w8.log 2>&1; rc=$?
echo "pytest w8 rc=$rc"; tail -1 $O/pytest_w8.log; [ $rc -ne 0 ] && exit $rc
for R in 1 2; do for L in libvpt_amd_base libvpt_amd libvpt_amd_w8; do
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 200 python tools/tune.py --spp 256 --gates 6:12:32:4 --reps 2 > $O/$L.$R.log 2>&1 || exit $?
  echo "c3 $L $(grep Msps $O/$L.$R.log | tail -1 | cut -c100-200)"
done; done
