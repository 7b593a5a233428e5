# gate_eval re-check with the final evaluation (C3)
export TMPDIR=/tmp; O=gpurun_out/r01aw; mkdir -p $O
timeout -k 10 400 python tools/tune.py --spp 256 --gates 8:12:32:4,8:12:28:4,8:12:36:4,8:12:24:4,8:12:32:4,6:12:32:4,8:12:32:4 --reps 2 > $O/tune.log 2>&1 || exit $?
grep Msps $O/tune.log | cut -c60-200
