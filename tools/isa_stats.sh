#!/bin/bash
# Register / scratch / occupancy summary of the integrator kernels (gfx950), plus the .s for reading.
# Usage: tools/isa_stats.sh [extra hipcc flags...]   -> /tmp/isa/vpt.s
mkdir -p /tmp/isa
R=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -I"$R/volume_path_tracer_amd/csrc" \
  --cuda-device-only -S -o /tmp/isa/vpt.s "$@" "$R/volume_path_tracer_amd/csrc/vpt_gpu.hip" 2>&1 | grep -v "unused during compilation"
python3 - <<'PY'
import re
t = open("/tmp/isa/vpt.s").read()
for m in re.finditer(r"^(_ZN3vpt20vpt_integrate_kernelI(\w+?)EEv\w*DevScene\w*):", t, re.M):
    seg = t[m.end():]
    get = lambda k: re.search(r"; %s: (\d+)" % k, seg).group(1)
    print(m.group(2), "vgpr", get("NumVgprs"), "sgpr", get("NumSGPRsForWavesPerEU"), "scratch", get("ScratchSize"), "occ", get("Occupancy"))
PY
