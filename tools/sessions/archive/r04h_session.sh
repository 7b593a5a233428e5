set -u
mkdir -p gpurun_out/r04h
timeout -k 10 300 python -u -m pytest tests/test_gpu_integration.py -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread -k "feed or stop_at or reference_signature or helper or share" > gpurun_out/r04h/pytest.log 2>&1 || { tail -40 gpurun_out/r04h/pytest.log; exit 1; }
tail -3 gpurun_out/r04h/pytest.log
bash tools/feed_diag.sh gpurun_out/r04h/fd
