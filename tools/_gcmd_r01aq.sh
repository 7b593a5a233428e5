# auto grid size for small launches: GPU tests, then bench C2 / C1 / C3
export TMPDIR=/tmp; O=gpurun_out/r01aq; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for C in c2 c1 c3; do
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 > $O/bench_$C.log 2>&1 || exit $?
  echo "$C $(tail -1 $O/bench_$C.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], (d.get("cpu_baseline") or {}).get("value"))')"
done
