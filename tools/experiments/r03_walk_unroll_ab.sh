# r03zv: the walk loop's exit check every 2 / 4 iterations (VPT_WALK_UNROLL) against the default 3, re-measured on the
# final r03 kernel: bench frames alternating default / variant (tools/ab_lib.sh; variants built with
# `python -m volume_path_tracer_amd.build --name=libvpt_u2.so -DVPT_WALK_UNROLL=2`, likewise u4)
set -o pipefail
PARITY=base bash tools/ab_lib.sh r03zv_u2 volume_path_tracer_amd/lib/libvpt_u2.so c3,c4 2 && bash tools/ab_lib.sh r03zv_u4 volume_path_tracer_amd/lib/libvpt_u4.so c3,c4 2
