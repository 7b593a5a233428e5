export TMPDIR=/tmp; O=gpurun_out/r01n; mkdir -p $O
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_prof.so timeout -k 10 300 python tools/tune.py --spp 64 --gates 8:8:16:4,8:8:16:0 --reps 1 --profile > $O/prof.log 2>&1 || exit $?
grep gate $O/prof.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-600
