#!/bin/bash
# A/B of a variant library build against the default one on the GPU box (timing + GPU parity):
# GPU production-parity tests (of the variant, or of the default build when PARITY=base), then bench.py
# frames of each config, alternating default / variant, <rounds> times.
#   python -m volume_path_tracer_amd.build --name=libvpt_exp.so -DVPT_EXP_...   (here, on the CPU)
#   bash tools/ab_lib.sh <tag> volume_path_tracer_amd/lib/libvpt_exp.so [configs=c3,c4] [rounds=2]
set -o pipefail
TAG=$1; VAR=$PWD/$2; CFGS=${3:-c3,c4}; ROUNDS=${4:-2}
BASE=$PWD/volume_path_tracer_amd/lib/libvpt_amd.so
O=gpurun_out/$TAG; mkdir -p $O
PL=$VAR; [ "${PARITY:-variant}" = base ] && PL=$BASE
VPT_LIB=$PL timeout -k 10 400 python -u -m pytest tests/test_gpu_production.py -x -q --timeout 120 --timeout-method thread > $O/pytest_${PARITY:-variant}.log 2>&1 || { tail -20 $O/pytest_${PARITY:-variant}.log; exit 1; }
tail -1 $O/pytest_${PARITY:-variant}.log
for r in $(seq 1 $ROUNDS); do
  for v in base variant; do
    L=$BASE; [ $v = variant ] && L=$VAR
    for c in ${CFGS//,/ }; do
      f=$O/b_${v}_${c}_$r
      VPT_LIB=$L timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > $f.json 2> $f.err || exit 1
      python -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$v $c $r', d['ms_per_step'], d['value'])"
    done
  done
done
