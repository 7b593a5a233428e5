# grid size when jobs < resident lanes: C2 (262144 jobs) and C1 (4096 jobs)
export TMPDIR=/tmp; O=gpurun_out/r01ap; mkdir -p $O
timeout -k 10 300 python tools/tune.py --config c2 --spp 64 --gates 8:12:32:4 --blocks 1792,1024,768,512,256 --reps 2 > $O/c2.log 2>&1 || exit $?
grep Msps $O/c2.log | cut -c60-200
timeout -k 10 300 python tools/tune.py --config c1 --spp 4 --gates 8:12:32:4 --blocks 1792,256,64,16 --reps 2 > $O/c1.log 2>&1 || exit $?
grep Msps $O/c1.log | cut -c60-200
