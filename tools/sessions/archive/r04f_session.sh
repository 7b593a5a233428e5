set -u
# Counter passes of C2 and C1 with the throughput kernel (--latency-kernel off) and the latency kernel
# (auto), then the C4 temperature-prefetch A/B (VPT_TEMP_PREFETCH=1 build, its production parity first).
bash tools/kernel_counters.sh r04f_thr c2 --latency-kernel off || exit 1
bash tools/kernel_counters.sh r04f_lat c2 --latency-kernel on || exit 1
bash tools/kernel_counters.sh r04f_thr c1 --latency-kernel off || exit 1
bash tools/kernel_counters.sh r04f_lat c1 --latency-kernel auto || exit 1
bash tools/ab_lib.sh r04f_tpre volume_path_tracer_amd/lib/libvpt_tpre.so c4 3 || exit 1
