# walk loop unrolled 2x (loop condition every second iteration): parity, A/B C3
export TMPDIR=/tmp; O=gpurun_out/r01ay; mkdir -p $O
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_u2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_u2.log 2>&1; rc=$?
echo "pytest u2 rc=$rc"; tail -1 $O/pytest_u2.log; [ $rc -ne 0 ] && exit $rc
for R in 1 2; do for L in libvpt_amd libvpt_amd_u2; do
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 200 python tools/tune.py --spp 256 --gates 6:12:32:4 --reps 2 > $O/$L.$R.log 2>&1 || exit $?
  echo "c3 $L $(grep Msps $O/$L.$R.log | tail -1 | cut -c100-200)"
done; done
