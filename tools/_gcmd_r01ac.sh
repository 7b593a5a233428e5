# compiler scheduling-strategy sweep (timing only; same source): default vs s1..s5
export TMPDIR=/tmp; O=gpurun_out/r01ac; mkdir -p $O
for L in libvpt_amd libvpt_amd_s1 libvpt_amd_s2 libvpt_amd_s3 libvpt_amd_s4 libvpt_amd_s5 libvpt_amd; do
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 200 python tools/tune.py --spp 256 --gates 8:12:32:4 --reps 2 > $O/$L.log 2>&1 || exit $?
  echo "$L $(grep Msps $O/$L.log | tail -1 | cut -c100-200)"
done
