# new GPU parity tests (C4 full-res job sample, fire_lowscattering) + C4 rocprof kernel stats
export TMPDIR=/tmp; O=gpurun_out/r01ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "c4_fullres or lowscattering" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/rocprof_c4.log 2>&1 || exit $?
tail -1 $O/rocprof_c4.log | cut -c1-300
find $O/prof_c4 -name "*stats*"
