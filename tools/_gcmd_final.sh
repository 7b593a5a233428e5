# round-end validation of the committed tree: GPU tests, smoke(), default bench
export TMPDIR=/tmp; O=gpurun_out/final; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-250
