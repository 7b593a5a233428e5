set -u
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_integration.py -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread -k "feed or stop_at or reference_signature or helper or share" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/feed_diag.sh $O/fd || exit 1
bash tools/drain_sweep.sh $O/drain || exit 1
bash tools/lat_ab.sh $O/lat || exit 1
bash tools/ab_probe.sh r04e/ab_r03 c3,c4 2 volume_path_tracer_amd/lib/libvpt_r03.so || exit 1
