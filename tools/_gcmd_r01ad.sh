# occupancy probe: same binary, persistent grid of 3/4/5 blocks per CU (256 CUs)
export TMPDIR=/tmp; O=gpurun_out/r01ad; mkdir -p $O
timeout -k 10 300 python tools/tune.py --spp 256 --gates 8:12:32:4 --blocks 768,1024,1280,1024,1280 --reps 2 > $O/blocks.log 2>&1 || exit $?
grep Msps $O/blocks.log | cut -c60-200
