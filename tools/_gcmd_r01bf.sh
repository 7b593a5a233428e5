# walk-loop exit when >= K lanes wait in the other states (VPT_GATE_OTHER), with the 3x-checked loop
export TMPDIR=/tmp; O=gpurun_out/r01bf; mkdir -p $O
for GO in 128 16 24 32 40 128; do
  VPT_GATE_OTHER=$GO timeout -k 10 200 python tools/tune.py --spp 256 --gates 6:12:32:4 --reps 2 > $O/go$GO.log 2>&1 || exit $?
  echo "go=$GO $(grep Msps $O/go$GO.log | tail -1 | cut -c100-200)"
done
