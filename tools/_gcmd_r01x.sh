export TMPDIR=/tmp; O=gpurun_out/r01x; mkdir -p $O
timeout -k 10 600 python tools/tune.py --spp 256 --gates 8:12:24:4,8:12:28:4,8:12:32:4,8:12:40:4,8:16:32:4,8:12:32:2,8:12:32:8,6:12:32:4,10:12:32:4 --reps 2 > $O/tune.log 2>&1 || exit $?
grep Msps $O/tune.log
