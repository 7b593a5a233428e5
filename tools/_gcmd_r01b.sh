export TMPDIR=/tmp; mkdir -p gpurun_out/r01b
( timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r01b/pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/r01b/pytest.log ) 
tail -3 gpurun_out/r01b/pytest.log
timeout -k 10 400 python tools/tune.py --spp 8 --gates 1:1,8:8,16:16,24:24,32:16,48:16 > gpurun_out/r01b/tune_default.log 2>&1 || exit $?
cat gpurun_out/r01b/tune_default.log | grep Msps
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_lb4.so timeout -k 10 400 python tools/tune.py --spp 8 --gates 1:1,16:16,32:16 > gpurun_out/r01b/tune_lb4.log 2>&1 || exit $?
cat gpurun_out/r01b/tune_lb4.log | grep Msps
