# r03zg record: parity of the chunked throughput mode, reference-mode A/B against the previous build
# (libvpt_prev.so = the sources before the change, built with `python -m volume_path_tracer_amd.build --name=libvpt_prev.so`
# from a checkout of them), and throughput-mode frames of C1 / C2 / C3.
set -o pipefail
O=gpurun_out/r03zg; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_throughput_mode.py tests/test_gpu_production.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_lib.sh r03zg volume_path_tracer_amd/lib/libvpt_prev.so c3,c4 2 > $O/ab_skip_parity.txt 2>&1 || true
for c in c1 c2 c3; do
  timeout -k 10 200 python bench.py --config $c --rng-mode pixel --steps 3 --warmup 1 --no-cpu-baseline > $O/pixel_$c.json 2> $O/pixel_$c.err || exit 1
  python -c "import json; d=json.loads(open('$O/pixel_$c.json').read().strip().splitlines()[-1]); print('pixel $c', d['ms_per_step'], d['value'])"
done
cat $O/ab_skip_parity.txt
