# separate gate for the heavy rare blocks (NEE completion, ray setup): VPT_GATE_HEAVY sweep (C3, C4)
export TMPDIR=/tmp; O=gpurun_out/r01bc; mkdir -p $O
for GH in 6 4 10 14 20 6; do
  VPT_GATE_HEAVY=$GH timeout -k 10 200 python tools/tune.py --spp 256 --gates 6:12:32:4 --reps 2 > $O/gh$GH.log 2>&1 || exit $?
  echo "c3 gh=$GH $(grep Msps $O/gh$GH.log | tail -1 | cut -c100-200)"
done
for GH in 6 12; do
  VPT_GATE_HEAVY=$GH timeout -k 10 200 python tools/tune.py --config c4 --spp 256 --gates 6:12:32:4 --reps 2 > $O/c4gh$GH.log 2>&1 || exit $?
  echo "c4 gh=$GH $(grep Msps $O/c4gh$GH.log | tail -1 | cut -c100-200)"
done
