#!/bin/bash
# r06a: the ordered film -- its GPU tests, the RCCL one-rank test, the production parity tests, then C3 / C4
# bench A/B (ordered vs atomic film), alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_multiprocess.py::test_rccl_one_rank_film_all_reduce \
  tests/test_gpu_film_order.py tests/test_gpu_production.py -x -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -8 $O/pytest.log; [ $rc -gt 1 ] && exit $rc
for C in c3 c4; do
  for m in ordered atomic ordered atomic; do
    timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-dropin --steps 5 --film-order $m >> $O/${C}_ab.jsonl 2>>$O/bench.err || exit 1
    tail -1 $O/${C}_ab.jsonl | cut -c1-200
  done
done
exit $rc
