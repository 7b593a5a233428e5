"""volume_path_tracer_amd — MI355X (gfx950) drop-in for the volume_path_tracer per-tile integrator.

Layers:
  include/vpt_gpu.h        C ABI (the drop-in boundary for vpt::run, src/worker.cpp:92-208)
  csrc/vpt_integrator.h    the device state machine (delta tracking, HDDA, NEE, blackbody)
  csrc/vpt_gpu.hip         persistent HIP kernels (throughput and latency variants) + context
  csrc/vpt_grid_build.cpp  NanoVDB-style grid -> HBM cell / walk tables + square-row stencil pool
  csrc/vpt_nanovdb.cpp     NanoGrid<float> memory and .nvdb files -> grid description
  csrc/vpt_config.cpp      strict scene-JSON reader (read_configuration)
  capi.py / scenes.py      ctypes mirror of the ABI, scene presets
  render.py                host driver: TileProvider-compatible job enumeration
  distributed.py           multi-GPU wave sharding and the RCCL film all-reduce
  include/vpt_run.hpp      the reference-side drop-in (vpt_gpu::run with vpt::run's signature)
"""
from . import capi  # noqa: F401

__all__ = ["capi"]
