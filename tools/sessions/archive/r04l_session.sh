set -u
mkdir -p gpurun_out/r04l
timeout -k 10 400 python -u -m pytest tests/test_gpu_production.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r04l/pytest_production.log 2>&1 || { tail -30 gpurun_out/r04l/pytest_production.log; exit 1; }
tail -1 gpurun_out/r04l/pytest_production.log
for C in c1 c2 c4; do
  timeout -k 10 300 python bench.py --config $C --steps 5 --warmup 1 --cpu-budget 6 > gpurun_out/r04l/bench_$C.json 2> gpurun_out/r04l/bench_$C.err || exit 1
  python3 -c "import json; j=json.loads(open('gpurun_out/r04l/bench_$C.json').read().strip().splitlines()[-1]); print('$C', j['ms_per_step'], j['value'])"
done
for S in 16 32; do
  timeout -k 10 300 python bench.py --config c3 --spp $S --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r04l/bench_c3s$S.json 2> gpurun_out/r04l/bench_c3s$S.err || exit 1
  python3 -c "import json; j=json.loads(open('gpurun_out/r04l/bench_c3s$S.json').read().strip().splitlines()[-1]); print('c3 spp $S', j['ms_per_step'], j['value'])"
done
timeout -k 10 600 python bench.py > gpurun_out/r04l/bench_c3.json 2> gpurun_out/r04l/bench_c3.err || exit 1
python3 -c "import json; j=json.loads(open('gpurun_out/r04l/bench_c3.json').read().strip().splitlines()[-1]); print('c3', j['ms_per_step'], j['value'])"
