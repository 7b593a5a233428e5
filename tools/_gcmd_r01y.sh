# gate_other sweep (default lib) + VPT_CIDX variant: parity on the variant, then timing
export TMPDIR=/tmp; O=gpurun_out/r01y; mkdir -p $O
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_cidx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_cidx.log 2>&1; rc=$?
echo "pytest cidx rc=$rc"; tail -2 $O/pytest_cidx.log; [ $rc -ne 0 ] && exit $rc
for GO in 64 16 24 32 40; do
  VPT_GATE_OTHER=$GO timeout -k 10 200 python tools/tune.py --spp 256 --gates 8:12:32:4 --reps 2 > $O/go$GO.log 2>&1 || exit $?
  echo "go=$GO $(grep Msps $O/go$GO.log | tail -1 | cut -c1-200)"
done
for L in libvpt_amd_cidx libvpt_amd; do
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 200 python tools/tune.py --spp 256 --gates 8:12:32:4 --reps 3 > $O/$L.log 2>&1 || exit $?
  echo "$L $(grep Msps $O/$L.log | tail -1 | cut -c1-200)"
done
