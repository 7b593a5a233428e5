# A/B timing of two library builds on one box (full C3 frame, default gates)
export TMPDIR=/tmp; O=gpurun_out/ab; mkdir -p $O
for L in ${LIBS:-libvpt_amd_base libvpt_amd}; do
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 300 python tools/tune.py --spp 256 --gates ${GATES:-8:12:24:4} --reps 3 > $O/$L.log 2>&1 || exit $?
  echo "$L $(grep Msps $O/$L.log | tail -1)"
done
