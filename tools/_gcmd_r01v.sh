export TMPDIR=/tmp; O=gpurun_out/r01v; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; if [ $rc -gt 1 ]; then exit $rc; fi
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd.so timeout -k 10 400 python tools/tune.py --spp 256 --gates 8:12:24:4 --reps 2 > $O/tune.log 2>&1 || exit $?
grep Msps $O/tune.log
