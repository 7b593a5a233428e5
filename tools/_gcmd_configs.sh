# bench lines for the other BASELINE configs (C1, C2, C4) on one GPU
export TMPDIR=/tmp; O=gpurun_out/configs; mkdir -p $O
for C in c4 c2 c1; do
  timeout -k 10 600 python bench.py --config $C --steps 2 --warmup 1 > $O/bench_$C.log 2>&1 || exit $?
  echo "$C $(tail -1 $O/bench_$C.log | cut -c1-300)"
done
timeout -k 10 400 python tools/tune.py --config c4 --spp 256 --gates 8:12:24:4,8:12:16:4,8:12:32:4,8:8:24:4 --reps 1 > $O/tune_c4.log 2>&1 || exit $?
grep Msps $O/tune_c4.log
