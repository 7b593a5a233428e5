# C4 gate sweep at 6 waves; throughput (pixel RNG) mode on C3 with the final kernel
export TMPDIR=/tmp; O=gpurun_out/r01ar; mkdir -p $O
timeout -k 10 400 python tools/tune.py --config c4 --spp 256 --gates 8:12:32:4,8:12:24:4,8:12:16:4,6:12:24:4,8:16:24:4,8:12:24:8,8:12:32:4 --reps 2 > $O/c4.log 2>&1 || exit $?
grep Msps $O/c4.log | cut -c60-200
timeout -k 10 300 python bench.py --rng-mode pixel --no-cpu-baseline > $O/bench_pixel.log 2>&1 || exit $?
tail -1 $O/bench_pixel.log | cut -c1-200
