export TMPDIR=/tmp; O=gpurun_out/r01m; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 $O/pytest.log
for L in libvpt_amd libvpt_amd_noint; do
VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 300 python tools/tune.py --spp 32 --gates 8:8:16:0,8:8:16:4,8:8:16:8,8:8:16:12,8:8:16:16,8:8:24:8,6:6:16:8 --reps 2 > $O/tune_$L.log 2>&1 || exit $?
grep Msps $O/tune_$L.log
done
