# gate sweep with the 3x-checked walk loop (C3)
export TMPDIR=/tmp; O=gpurun_out/r01ba; mkdir -p $O
timeout -k 10 500 python tools/tune.py --spp 256 --gates 6:12:32:4,6:12:36:4,6:12:40:4,6:12:32:2,6:12:32:8,6:16:32:4,6:8:32:4,8:12:32:4,6:12:32:4 --reps 2 > $O/tune.log 2>&1 || exit $?
grep Msps $O/tune.log | cut -c60-200
