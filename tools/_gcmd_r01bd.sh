# temperature sampler cell in LDS for the temperature kernel: parity, A/B C3 + C4
export TMPDIR=/tmp; O=gpurun_out/r01bd; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for R in 1 2; do for L in libvpt_amd_base libvpt_amd; do
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 200 python tools/tune.py --spp 256 --gates 6:12:32:4 --reps 2 > $O/$L.$R.log 2>&1 || exit $?
  echo "c3 $L $(grep Msps $O/$L.$R.log | tail -1 | cut -c100-200)"
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 200 python tools/tune.py --config c4 --spp 256 --gates 6:12:32:4 --reps 2 > $O/$L.c4.$R.log 2>&1 || exit $?
  echo "c4 $L $(grep Msps $O/$L.c4.$R.log | tail -1 | cut -c100-200)"
done; done
