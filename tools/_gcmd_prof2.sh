#!/bin/bash
# A/B of the default library vs base, then the SIMT census (VPT_PROFILE) and section cycles
# (VPT_PROFILE_TIME) of the full C3 frame at the default gates.
export TMPDIR=/tmp; O=gpurun_out/${1:-prof4}; mkdir -p $O
G=${GATES:-8:12:32:4}
for L in libvpt_amd_base libvpt_amd; do
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 300 python tools/tune.py --spp 256 --gates $G --reps 2 > $O/$L.log 2>&1 || exit $?
  echo "$L $(grep Msps $O/$L.log | tail -1 | cut -c60-200)"
done
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_prof.so timeout -k 10 300 python tools/tune.py --spp 64 --gates $G --reps 1 --profile > $O/prof.log 2>&1 || exit $?
grep profile $O/prof.log | cut -c1-1500
VPT_LIB=$PWD/volume_path_tracer_amd/lib/libvpt_amd_ptime.so timeout -k 10 300 python tools/tune.py --spp 256 --gates $G --reps 1 --profile > $O/ptime.log 2>&1 || exit $?
grep cycles $O/ptime.log | python3 -c "import sys,json; [print(json.loads(l)['profile']['cycles'], json.loads(l)['profile']['cycles_total']) for l in sys.stdin if 'profile' in l]"
