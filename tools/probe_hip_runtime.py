"""Probe (tools only, GPU box): one HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 /
libhsa-runtime64; libvpt_amd.so links /opt/rocm's.  Whichever loads first serves both (same sonames) --
unless /opt/rocm's comes first, then torch loads its own second ROCr, which on some boxes finds no GPU.
    python tools/probe_hip_runtime.py raw_vpt_first   # ctypes.CDLL(libvpt_amd.so), then torch: may fail
    python tools/probe_hip_runtime.py capi            # capi.lib() (imports torch first), then torch: ok
Prints the runtimes mapped into the process and whether a torch tensor and an Integrator work."""
import ctypes
import sys

sys.path.insert(0, ".")
mode = sys.argv[1]
if mode == "raw_vpt_first":
    ctypes.CDLL("volume_path_tracer_amd/lib/libvpt_amd.so")
from volume_path_tracer_amd.scenes import SynthGrid, workload  # noqa: E402

wl = workload("c3", width=32, height=24, spp=16, grid_n=64)
dens = SynthGrid(wl.density_kind, wl.grid_n).grid()  # capi.lib()
import torch  # noqa: E402

libs = sorted({ln.split()[-1] for ln in open("/proc/self/maps") if "amdhip64" in ln or "hsa-runtime" in ln})
try:
    from volume_path_tracer_amd.render import Integrator

    it = Integrator(wl.cfg, dens, None, device=0)
    torch.zeros(4, device="cuda")
    torch.cuda.synchronize()
    print(mode, "ok", libs)
except Exception as e:  # noqa: BLE001
    print(mode, "FAIL", e, libs)
