export TMPDIR=/tmp; O=gpurun_out/r01d; mkdir -p $O
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_prof.so timeout -k 10 300 python tools/tune.py --spp 8 --gates 1:1,8:8,16:16 --reps 1 --profile > $O/prof.log 2>&1; echo rc=$?
grep -v Warn $O/prof.log | tail -8
