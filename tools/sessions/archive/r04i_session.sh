set -u
# Final-binary check after the drain's push batches and the compaction code's removal: every GPU test + smoke,
# then the drain sweep (push_batch / cost_order A/B, C4 with and without push batches).
STEPS="pytest smoke" bash tools/gpu_check.sh r04i/check || exit 1
grep -q "passed" gpurun_out/r04i/check/pytest_gpu.log && ! grep -q "failed" gpurun_out/r04i/check/pytest_gpu.log || { tail -20 gpurun_out/r04i/check/pytest_gpu.log; exit 1; }
bash tools/drain_sweep.sh gpurun_out/r04i/drain || exit 1
