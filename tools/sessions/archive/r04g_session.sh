set -u
# Live-path compaction (tools/experiments/r04_compaction.patch applied, built with -DVPT_EXP_COMPACT=8 / 32 as
# libvpt_cmp8.so / libvpt_cmp32.so, and a 5-wave production build libvpt_w5.so) measured: its production parity, then C3 frames of the production
# binary (7 waves), the same kernel at 5 waves (the compaction build's occupancy) and compaction every 8 / 32
# outer iterations at 5 waves; then SQ / memory counters of the 5-wave baseline and compaction every 8.
L=$PWD/volume_path_tracer_amd/lib
bash tools/ab_lib.sh r04g_cmp8 volume_path_tracer_amd/lib/libvpt_cmp8.so c3 2 || exit 1
bash tools/ab_probe.sh r04g_probe c3 2 $L/libvpt_w5.so $L/libvpt_cmp32.so || exit 1
VPT_LIB=$L/libvpt_w5.so bash tools/kernel_counters.sh r04g_w5 c3 || exit 1
VPT_LIB=$L/libvpt_cmp8.so bash tools/kernel_counters.sh r04g_cmp8 c3 || exit 1
