# bench lines for the other BASELINE configs on one GPU (C4 fire, C2 homogeneous, C1 small, C5 frame on 1 GPU)
export TMPDIR=/tmp; O=gpurun_out/configs2; mkdir -p $O
for C in c4 c2 c1; do
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 > $O/bench_$C.log 2>&1 || exit $?
  echo "$C $(tail -1 $O/bench_$C.log | cut -c1-400)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/rocprof_c4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit $?
echo "c5 $(tail -1 $O/bench_c5.log | cut -c1-400)"
