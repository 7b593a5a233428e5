# SIMT census (VPT_PROFILE) and section cycles (VPT_PROFILE_TIME) of the 7-wave kernel, C3 256 spp
export TMPDIR=/tmp; O=gpurun_out/r01an; mkdir -p $O
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_prof.so timeout -k 10 300 python tools/tune.py --spp 256 --gates 8:12:32:4 --reps 1 --profile > $O/prof.log 2>&1 || exit $?
grep profile $O/prof.log | cut -c1-2500
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_ptime.so timeout -k 10 300 python tools/tune.py --spp 256 --gates 8:12:32:4 --reps 1 --profile > $O/ptime.log 2>&1 || exit $?
grep cycles $O/ptime.log | python3 -c "import sys,json; [print(json.loads(l)['profile']['cycles'], json.loads(l)['profile']['cycles_total']) for l in sys.stdin if 'profile' in l]"
