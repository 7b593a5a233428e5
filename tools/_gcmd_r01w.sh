export TMPDIR=/tmp; O=gpurun_out/r01w; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python tools/tune.py --spp 256 --gates 8:12:24:4 --reps 1 > $O/tune_ref.log 2>&1 || exit $?
grep Msps $O/tune_ref.log
timeout -k 10 400 python tools/tune.py --spp 256 --gates 8:12:24:4,8:12:16:4,8:12:32:4 --reps 1 --rng-mode pixel > $O/tune_pix.log 2>&1 || exit $?
grep Msps $O/tune_pix.log
