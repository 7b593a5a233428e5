# 6 waves/SIMD (launch bounds; 80 VGPRs with some spills) vs 5
export TMPDIR=/tmp; O=gpurun_out/r01ae; mkdir -p $O
for L in libvpt_amd libvpt_amd_w6 libvpt_amd libvpt_amd_w6; do
  VPT_LIB=$PWD/volume_path_tracer_amd/lib/$L.so timeout -k 10 200 python tools/tune.py --spp 256 --gates 8:12:32:4 --reps 2 > $O/$L.log 2>&1 || exit $?
  echo "$L $(grep Msps $O/$L.log | tail -1 | cut -c100-200)"
done
