# walk-loop unroll 2/3/4: parity of u4, A/B C3 (+ gate_eval 24/28 with u2), C4 with u2
export TMPDIR=/tmp; O=gpurun_out/r01az; mkdir -p $O
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_u4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_u4.log 2>&1; rc=$?
echo "pytest u4 rc=$rc"; tail -1 $O/pytest_u4.log; [ $rc -ne 0 ] && exit $rc
for L in libvpt_amd libvpt_amd_u2 libvpt_amd_u3 libvpt_amd_u4; do
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 200 python tools/tune.py --spp 256 --gates 6:12:32:4,6:12:28:4,6:12:24:4 --reps 2 > $O/$L.log 2>&1 || exit $?
  grep Msps $O/$L.log | sed "s/^/$L /" | cut -c1-20,120-200
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 200 python tools/tune.py --config c4 --spp 256 --gates 6:12:32:4 --reps 2 > $O/$L.c4.log 2>&1 || exit $?
  echo "c4 $L $(grep Msps $O/$L.c4.log | tail -1 | cut -c100-200)"
done
