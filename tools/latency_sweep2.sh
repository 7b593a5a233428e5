#!/bin/bash
# Latency-launch threshold: C1 frames of 4..64 spp (4 096..65 536 jobs), spread over the full grid
# (default latency knobs) vs the 256-block, 64-lane sizing with the throughput gates.
set -u
export TMPDIR=/tmp; O=gpurun_out/${1:-lat}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_production.py -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; if [ $rc -ne 0 ]; then tail -30 $O/pytest.log; exit $rc; fi
for S in 4 8 16 32 48 64; do
  timeout -k 10 300 python tools/tune.py --config c1 --spp $S --gates 6:8:36:4 --blocks 1792 --reps 3 > $O/c1_s$S.log 2>&1 || exit 1
  timeout -k 10 300 python tools/tune.py --config c1 --spp $S --gates 6:8:36:4 --blocks 256 --lat 64:6:8:36:4 --reps 3 >> $O/c1_s$S.log 2>&1 || exit 1
  grep Msps $O/c1_s$S.log | grep -o '"lat".*'
done
timeout -k 10 300 python bench.py --config c1 --steps 5 --warmup 2 --cpu-budget 3 > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
cat $O/bench_c1.json | cut -c1-400
timeout -k 10 300 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
cat $O/bench_c2.json | cut -c1-400
