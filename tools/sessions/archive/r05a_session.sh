#!/bin/bash
# r05a: copies beside a persistent kernel (SDMA probe), the r04 drop-in's drain (no switch / 0.2-s film) and
# the one-launch C3 frame in jid order vs the cost-tail order -- the drop-in gap decomposed.
set -eu
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 60 tools/ubench/sdma_probe 32 1000 > $O/sdma.txt 2>&1; cat $O/sdma.txt
timeout -k 10 60 tools/ubench/sdma_probe 128 1000 >> $O/sdma.txt 2>&1; tail -7 $O/sdma.txt
H=tests/native/build/run_gpu_harness
for r in 1 2; do
  for f in 100000 200; do
    timeout -k 10 120 $H config=volume_path_tracer_amd/scenes/wdas_cloud.json out=$O/film.f32 w=1920 h=1080 waves=256 \
      grid_n=512 threads=1 batch=4096 flush_ms=$f > $O/drain_f$f.log 2>&1
    echo "drain flush_ms=$f $(grep render_ms $O/drain_f$f.log)"
  done
done
rm -f $O/film.f32
timeout -k 10 300 python tools/tune.py --config c3 --spp 256 --gates 6:8:36:4 --order 0 --reps 2 > $O/order.jsonl 2>$O/order.err
timeout -k 10 300 python tools/tune.py --config c3 --spp 256 --gates 6:8:36:4 --order 3 --reps 2 >> $O/order.jsonl 2>>$O/order.err
cat $O/order.jsonl
