# fire (C4) kernel occupancy: natural 5 waves vs launch bounds 6 / 7; C3 gate_min 6 vs 8
export TMPDIR=/tmp; O=gpurun_out/r01aj; mkdir -p $O
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_t7.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "c4 or lowscattering" > $O/pytest_t7.log 2>&1; rc=$?
echo "pytest t7 rc=$rc"; tail -1 $O/pytest_t7.log; [ $rc -ne 0 ] && exit $rc
for R in 1 2; do for L in libvpt_amd libvpt_amd_t6 libvpt_amd_t7; do
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 200 python tools/tune.py --config c4 --spp 256 --gates 8:12:32:4 --reps 2 > $O/$L.$R.log 2>&1 || exit $?
  echo "c4 $L $(grep Msps $O/$L.$R.log | tail -1 | cut -c100-200)"
done; done
timeout -k 10 300 python tools/tune.py --spp 256 --gates 8:12:32:4,6:12:32:4,5:12:32:4,6:10:32:4,6:12:28:4,8:12:32:4,6:12:32:4 --reps 2 > $O/gates.log 2>&1 || exit $?
grep Msps $O/gates.log | cut -c60-200
