# gate re-tuning at 7 waves/SIMD (C3, 256 spp)
export TMPDIR=/tmp; O=gpurun_out/r01ah; mkdir -p $O
timeout -k 10 500 python tools/tune.py --spp 256 --gates 8:12:32:4,8:12:24:4,8:12:40:4,8:12:48:4,8:16:32:4,8:8:32:4,6:12:32:4,12:12:32:4,8:12:32:2,8:12:32:8,8:12:32:4 --reps 2 > $O/tune.log 2>&1 || exit $?
grep Msps $O/tune.log | cut -c60-200
