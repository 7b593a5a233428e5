# quick GPU check: parity tests + full-frame C3 timing (2 reps) at the default gates
export TMPDIR=/tmp; O=gpurun_out/quick; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python tools/tune.py --spp 256 --gates ${GATES:-8:12:24:4} --reps 2 > $O/tune.log 2>&1 || exit $?
grep Msps $O/tune.log
