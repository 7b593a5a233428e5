# job-order tail length at 7 waves (auto = 6 x resident lanes / T = 85 waves of 256)
export TMPDIR=/tmp; O=gpurun_out/r01al; mkdir -p $O
for TL in 0 40 60 110 140 0; do
  timeout -k 10 200 python tools/tune.py --spp 256 --gates 8:12:32:4 --reps 2 --tail $TL > $O/t$TL.log 2>&1 || exit $?
  echo "tail=$TL $(grep Msps $O/t$TL.log | tail -1 | cut -c100-200)"
done
