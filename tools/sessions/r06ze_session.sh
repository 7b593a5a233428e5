#!/bin/bash
# r06ze: the same-tile job order as the default (VPT_ORDER_COST_SAME_TILE): its GPU parity (production, ordered
# film, job orders), then bench frames against the previous default (libvpt_tail.so: VPT_ORDER_COST_TAIL) on C1-C4,
# the C3 8-GPU share (32 waves) on both, and the strong-scaling emulation on the new default.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06ze; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_film_order.py tests/test_gpu_order.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -20 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
bash tools/ab_multi.sh r06ze "tail" c3,c4,c2,c1 2 || exit $?
for v in base tail; do
  L=$PWD/volume_path_tracer_amd/lib/libvpt_amd.so; [ $v = tail ] && L=$PWD/volume_path_tracer_amd/lib/libvpt_tail.so
  for r in 1 2; do
    VPT_LIB=$L timeout -k 10 200 python bench.py --config c3 --spp 32 --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $O/share32_${v}_$r.json 2> $O/share32_${v}_$r.err || exit 1
    echo "share32 $v $r $(grep -o '"ms_per_step": [0-9.]*' $O/share32_${v}_$r.json)" | tee -a $O/summary.txt
  done
done
bash tools/strong_emulation.sh r06ze_strong || exit $?
