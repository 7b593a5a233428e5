export TMPDIR=/tmp; O=gpurun_out/r01u; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; if [ $rc -gt 1 ]; then exit $rc; fi
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd.so timeout -k 10 400 python tools/tune.py --spp 256 --gates 8:12:24:4:8,8:12:24:4:4,8:12:24:4:16,8:12:24:4:1,8:12:24:4:24 --reps 1 > $O/tune.log 2>&1 || exit $?
grep Msps $O/tune.log
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_prof.so timeout -k 10 400 python tools/tune.py --spp 64 --gates 8:12:24:4:8 --reps 1 --profile > $O/prof.log 2>&1 || exit $?
grep profile $O/prof.log | cut -c1-900
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_ptime.so timeout -k 10 300 python tools/tune.py --spp 256 --gates 8:12:24:4:8 --reps 1 --profile > $O/ptime.log 2>&1 || exit $?
grep cycles $O/ptime.log | python3 -c "import sys,json; [print(json.loads(l)['gate'], json.loads(l)['profile']['cycles']) for l in sys.stdin]"
