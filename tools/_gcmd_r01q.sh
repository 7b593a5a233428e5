export TMPDIR=/tmp; O=gpurun_out/r01q; mkdir -p $O
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_ptime.so timeout -k 10 300 python tools/tune.py --spp 256 --gates 8:12:24:4 --reps 1 --profile > $O/ptime.log 2>&1 || exit $?
grep cycles $O/ptime.log | python3 -c "import sys,json; [print(json.loads(l)['gate'], json.loads(l)['profile']['cycles']) for l in sys.stdin]"
for L in libvpt_amd libvpt_amd_ablog libvpt_amd_abdiv; do
VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 300 python tools/tune.py --spp 256 --gates 8:12:24:4 --reps 1 > $O/tune_$L.log 2>&1 || exit $?
grep Msps $O/tune_$L.log
done
