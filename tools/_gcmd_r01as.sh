# run-skipping kernel variant (auto for C2): GPU tests, parity of the forced variant on the cloud,
# A/B on C2 and C3 (VPT_RUNS forces the variant)
export TMPDIR=/tmp; O=gpurun_out/r01as; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
VPT_RUNS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_runs1.log 2>&1; rc=$?
echo "pytest VPT_RUNS=1 rc=$rc"; tail -1 $O/pytest_runs1.log; [ $rc -ne 0 ] && exit $rc
for R in 1 2; do
  for V in 0 1; do
    VPT_RUNS=$V timeout -k 10 200 python bench.py --config c2 --no-cpu-baseline > $O/c2.$V.$R.log 2>&1 || exit $?
    echo "c2 runs=$V $(tail -1 $O/c2.$V.$R.log | cut -c90-140)"
    VPT_RUNS=$V timeout -k 10 200 python tools/tune.py --spp 256 --gates 8:12:32:4 --reps 2 > $O/c3.$V.$R.log 2>&1 || exit $?
    echo "c3 runs=$V $(grep Msps $O/c3.$V.$R.log | tail -1 | cut -c100-200)"
  done
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_base.so timeout -k 10 200 python tools/tune.py --spp 256 --gates 8:12:32:4 --reps 2 > $O/c3.base.$R.log 2>&1 || exit $?
  echo "c3 base $(grep Msps $O/c3.base.$R.log | tail -1 | cut -c100-200)"
done
