"""ctypes mirror of include/vpt_gpu.h (the C ABI of the HIP integrator) and library loading.

The product library is ``volume_path_tracer_amd/lib/libvpt_amd.so`` (HIP, gfx950), built in-tree by
``__graft_entry__.build()``.  There is no fallback: if it is missing, importing a GPU entry point
raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
LIB_DIR = PKG_DIR / "lib"
LIB_PATH = Path(os.environ["VPT_LIB"]) if os.environ.get("VPT_LIB") else LIB_DIR / "libvpt_amd.so"

VPT_OK = 0
VPT_BLACKBODY_ROWS = 500


class CameraParams(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("look", C.c_float * 3), ("up", C.c_float * 3),
                ("vfov_deg", C.c_float), ("imaging_ratio", C.c_float)]


class WorkerParams(C.Structure):
    _fields_ = [("single_pixel_enabled", C.c_int32), ("use_jitter", C.c_int32),
                ("single_pixel_coord", C.c_int64 * 2),
                ("infinite_light_xyz", C.c_float * 3), ("infinite_light_multiplier", C.c_float),
                ("distant_light_xyz", C.c_float * 3), ("distant_light_multiplier", C.c_float),
                ("distant_light_inv_direction", C.c_float * 3), ("max_depth", C.c_uint32)]


class VolumeParams(C.Structure):
    _fields_ = [("henyey_greenstein_g", C.c_float), ("le_scale", C.c_float), ("sigma_a", C.c_float),
                ("sigma_s", C.c_float), ("temperature_offset", C.c_float), ("temperature_scale", C.c_float)]


class Configuration(C.Structure):
    """include/vpt/configuration.hpp:61-71 (vpt_configuration)."""
    _fields_ = [("seed", C.c_uint32), ("num_waves", C.c_uint32), ("num_workers", C.c_uint32),
                ("_pad0", C.c_uint32),
                ("output_size", C.c_int64 * 2), ("tile_size", C.c_int64 * 2),
                ("camera_parameters", CameraParams), ("worker_parameters", WorkerParams),
                ("volume_parameters", VolumeParams), ("volume_path", C.c_char * 4096)]

    def copy(self) -> "Configuration":
        c = Configuration()
        C.memmove(C.byref(c), C.byref(self), C.sizeof(Configuration))
        return c

    @property
    def width(self) -> int:
        return int(self.output_size[0])

    @property
    def height(self) -> int:
        return int(self.output_size[1])

    def jobs_per_wave(self) -> int:
        tw, th = int(self.tile_size[0]), int(self.tile_size[1])
        return (-(-self.width // tw)) * (-(-self.height // th))


class GridDesc(C.Structure):
    """vpt_grid_desc: a NanoVDB float grid flattened to arrays (volume_grids.hpp:12-14)."""
    _fields_ = [("map_mat", C.c_float * 9), ("map_inv_mat", C.c_float * 9), ("map_vec", C.c_float * 3),
                ("background", C.c_float),
                ("index_bbox_min", C.c_int32 * 3), ("index_bbox_max", C.c_int32 * 3),
                ("leaf_count", C.c_uint64),
                ("leaf_origin", C.POINTER(C.c_int32)), ("leaf_values", C.POINTER(C.c_float)),
                ("leaf_value_mask", C.POINTER(C.c_uint64)), ("leaf_max", C.POINTER(C.c_float)),
                ("tile_count", C.c_uint64),
                ("tile_origin", C.POINTER(C.c_int32)), ("tile_level", C.POINTER(C.c_int32)),
                ("tile_value", C.POINTER(C.c_float)), ("tile_active", C.POINTER(C.c_uint8)),
                ("lower_count", C.c_uint64), ("lower_origin", C.POINTER(C.c_int32)),
                ("upper_count", C.c_uint64), ("upper_origin", C.POINTER(C.c_int32))]


class Counters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("samples", "dda_steps", "segments", "draws", "stencils",
                                          "density_evals", "temp_stencils", "scatters", "shadow_rays",
                                          "rng_draws", "exchanged")]

    def as_dict(self) -> dict:
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


# vpt_event (include/vpt_gpu.h): one Logger line (src/worker.cpp:16-48)
EVENT_DTYPE = np.dtype([("jid", "<u8"), ("pixel", "<u4"), ("seq", "<u4"), ("type", "<u4"), ("v", "<f4", (7,))])
assert EVENT_DTYPE.itemsize == 48
# vpt_dda_row (Volume::log_dda_trace, one dda_trace.csv line)
DDA_ROW_DTYPE = np.dtype([("ijk", "<i4", (3,)), ("t", "<f4"), ("value", "<f4"), ("dim_getdim", "<u4"),
                          ("dim_nodeinfo", "<u4"), ("active", "<i4"), ("maximum", "<f4")])
assert DDA_ROW_DTYPE.itemsize == 36
VPT_RNG_REFERENCE, VPT_RNG_PIXEL = 0, 1
VPT_ORDER_JID, VPT_ORDER_COST_WAVE_MAJOR, VPT_ORDER_COST_TILE_MAJOR, VPT_ORDER_COST_TAIL = 0, 1, 2, 3
VPT_ORDER_COST_SAME_TILE = 4
VPT_FILM_ATOMIC, VPT_FILM_ORDERED = 0, 1
EVENT_NAMES = ("new_ray", "sampled_point", "null", "scatter_terminated", "scatter", "absorbed")


def _ptr(arr, ctype):
    if arr is None:
        return C.cast(None, C.POINTER(ctype))
    return arr.ctypes.data_as(C.POINTER(ctype))


class Grid:
    """A grid held as numpy arrays plus the GridDesc view of them (keeps the arrays alive)."""

    def __init__(self, *, map_mat, map_inv_mat, map_vec, background, bbox_min, bbox_max,
                 leaf_origin, leaf_values, leaf_max, leaf_value_mask=None,
                 tile_origin=None, tile_level=None, tile_value=None, tile_active=None,
                 lower_origin=None, upper_origin=None):
        self.leaf_origin = np.ascontiguousarray(leaf_origin, dtype=np.int32).reshape(-1, 3)
        n = self.leaf_origin.shape[0]
        self.leaf_values = np.ascontiguousarray(leaf_values, dtype=np.float32).reshape(n, 512)
        self.leaf_max = np.ascontiguousarray(leaf_max, dtype=np.float32).reshape(n)
        if leaf_value_mask is None:
            leaf_value_mask = np.full((n, 8), np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
        self.leaf_value_mask = np.ascontiguousarray(leaf_value_mask, dtype=np.uint64).reshape(n, 8)
        self.tile_origin = None if tile_origin is None else np.ascontiguousarray(tile_origin, dtype=np.int32).reshape(-1, 3)
        self.tile_level = None if tile_level is None else np.ascontiguousarray(tile_level, dtype=np.int32)
        self.tile_value = None if tile_value is None else np.ascontiguousarray(tile_value, dtype=np.float32)
        self.tile_active = None if tile_active is None else np.ascontiguousarray(tile_active, dtype=np.uint8)
        self.lower_origin = None if lower_origin is None else np.ascontiguousarray(lower_origin, dtype=np.int32).reshape(-1, 3)
        self.upper_origin = None if upper_origin is None else np.ascontiguousarray(upper_origin, dtype=np.int32).reshape(-1, 3)
        d = GridDesc()
        d.map_mat[:] = [float(x) for x in np.asarray(map_mat, dtype=np.float32).reshape(9)]
        d.map_inv_mat[:] = [float(x) for x in np.asarray(map_inv_mat, dtype=np.float32).reshape(9)]
        d.map_vec[:] = [float(x) for x in np.asarray(map_vec, dtype=np.float32).reshape(3)]
        d.background = float(np.float32(background))
        d.index_bbox_min[:] = [int(x) for x in bbox_min]
        d.index_bbox_max[:] = [int(x) for x in bbox_max]
        d.leaf_count = n
        d.leaf_origin = _ptr(self.leaf_origin, C.c_int32)
        d.leaf_values = _ptr(self.leaf_values, C.c_float)
        d.leaf_value_mask = _ptr(self.leaf_value_mask, C.c_uint64)
        d.leaf_max = _ptr(self.leaf_max, C.c_float)
        d.tile_count = 0 if self.tile_origin is None else self.tile_origin.shape[0]
        d.tile_origin = _ptr(self.tile_origin, C.c_int32)
        d.tile_level = _ptr(self.tile_level, C.c_int32)
        d.tile_value = _ptr(self.tile_value, C.c_float)
        d.tile_active = _ptr(self.tile_active, C.c_uint8)
        d.lower_count = 0 if self.lower_origin is None else self.lower_origin.shape[0]
        d.lower_origin = _ptr(self.lower_origin, C.c_int32)
        d.upper_count = 0 if self.upper_origin is None else self.upper_origin.shape[0]
        d.upper_origin = _ptr(self.upper_origin, C.c_int32)
        self.desc = d

    @classmethod
    def from_desc(cls, d: GridDesc, copy: bool = True) -> "Grid":
        n = int(d.leaf_count)

        def arr(p, shape, dt):
            if not p or int(np.prod(shape)) == 0:
                return None
            a = np.ctypeslib.as_array(p, shape=shape)
            return a.astype(dt, copy=True) if copy else a

        t = int(d.tile_count)
        return cls(map_mat=list(d.map_mat), map_inv_mat=list(d.map_inv_mat), map_vec=list(d.map_vec),
                   background=d.background, bbox_min=list(d.index_bbox_min), bbox_max=list(d.index_bbox_max),
                   leaf_origin=arr(d.leaf_origin, (n, 3), np.int32) if n else np.zeros((0, 3), np.int32),
                   leaf_values=arr(d.leaf_values, (n, 512), np.float32) if n else np.zeros((0, 512), np.float32),
                   leaf_max=arr(d.leaf_max, (n,), np.float32) if n else np.zeros((0,), np.float32),
                   leaf_value_mask=arr(d.leaf_value_mask, (n, 8), np.uint64) if n else None,
                   tile_origin=arr(d.tile_origin, (t, 3), np.int32), tile_level=arr(d.tile_level, (t,), np.int32),
                   tile_value=arr(d.tile_value, (t,), np.float32), tile_active=arr(d.tile_active, (t,), np.uint8),
                   lower_origin=arr(d.lower_origin, (int(d.lower_count), 3), np.int32),
                   upper_origin=arr(d.upper_origin, (int(d.upper_count), 3), np.int32))

    @property
    def leaf_count(self) -> int:
        return int(self.leaf_origin.shape[0])


def load_cie(path: Path | None = None):
    """CIE 1931 table shipped with the package -> (float32[471,3], float32 Y_integral).

    Values are parsed as doubles then rounded to float, exactly like the reference's
    constexpr std::array<float> initialisers (src/spectral_data/xyz.hpp:17,116,215,314)."""
    path = path or (PKG_DIR / "data" / "cie1931_xyz.csv")
    rows, yint = [], None
    for line in Path(path).read_text().splitlines():
        if line.startswith("# Y_integral="):
            yint = np.float32(float(line.split("=", 1)[1]))
        elif line and not line.startswith("#") and not line.startswith("lambda"):
            rows.append([float(v) for v in line.split(",")[1:]])
    cie = np.asarray(rows, dtype=np.float64).astype(np.float32)
    assert cie.shape == (471, 3) and yint is not None
    return np.ascontiguousarray(cie), yint


_lib = None


def lib() -> C.CDLL:
    """The HIP integrator library; raises if it has not been built (no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc, gfx950)")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64.  Loaded first,
    # they also serve this library (same sonames), and the device memory torch allocates is the memory the
    # kernels see.  Loaded after /opt/rocm's (this library's link-time runtime), torch's ROCr opens the GPU a
    # second time and, on some boxes, finds none ("No HIP GPUs are available"; r03zl,
    # tools/probe_hip_init2.py).  So torch is imported before the library, whatever the caller imported.
    # Host-only uses (grid readers, the C-ABI host tests) need no torch: without it there is no second runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(str(LIB_PATH))
    cfgp, gridp = C.POINTER(Configuration), C.POINTER(GridDesc)
    fp, vp = C.POINTER(C.c_float), C.c_void_p
    L.vpt_config_read.argtypes = [C.c_char_p, cfgp]
    L.vpt_config_parse.argtypes = [C.c_char_p, C.c_size_t, cfgp]
    L.vpt_fix_majorants.argtypes = [gridp, fp, C.c_int]
    L.vpt_blackbody_table.argtypes = [fp]
    L.vpt_blackbody_xyz.argtypes = [fp, C.c_float, fp]
    L.vpt_gpu_create.argtypes = [cfgp, gridp, gridp, fp, C.c_int, C.POINTER(vp)]
    if hasattr(L, "vpt_gpu_create_many"):
        L.vpt_gpu_create_many.argtypes = [cfgp, gridp, gridp, fp, C.POINTER(C.c_int), C.c_int, C.POINTER(vp)]
    if hasattr(L, "vpt_gpu_frame_open"):
        L.vpt_gpu_frame_open.argtypes = [vp, C.c_uint64, C.POINTER(C.c_uint64), C.c_uint32, C.c_uint32]
        L.vpt_gpu_frame_finish.argtypes = [vp, C.c_uint64, fp, fp]
    if hasattr(L, "vpt_grids_flatten"):
        L.vpt_grids_flatten.argtypes = [gridp, gridp, C.POINTER(vp)]
        L.vpt_gpu_create_from.argtypes = [cfgp, vp, fp, C.POINTER(C.c_int), C.c_int, C.POINTER(vp)]
        L.vpt_grids_free.argtypes = [vp]
        L.vpt_grids_free.restype = None
    L.vpt_gpu_destroy.argtypes = [vp]
    L.vpt_gpu_job_space.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.vpt_gpu_render_jobs.argtypes = [vp, C.c_uint64, C.c_uint64, vp, vp]
    L.vpt_gpu_render_jobs_records.argtypes = [vp, C.c_uint64, C.c_uint64, vp, vp, vp]
    L.vpt_gpu_sync.argtypes = [vp]
    L.vpt_gpu_film_clear.argtypes = [vp]
    L.vpt_gpu_film_device_ptr.argtypes = [vp, C.POINTER(vp), C.POINTER(C.c_uint64)]
    L.vpt_gpu_film_add_to_host.argtypes = [vp, fp]
    L.vpt_gpu_counters.argtypes = [vp, C.POINTER(Counters), C.c_int]
    L.vpt_gpu_profile.argtypes = [vp, C.POINTER(C.c_uint64), C.c_int, C.c_int]
    L.vpt_gpu_set_tuning.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    if hasattr(L, "vpt_gpu_set_latency_tuning"):  # (older builds in A/B runs lack it)
        L.vpt_gpu_set_latency_tuning.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    L.vpt_gpu_launch_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.vpt_last_error.restype = C.c_char_p
    L.vpt_synth_grid.argtypes = [C.c_int, C.c_int]
    L.vpt_synth_grid.restype = gridp
    L.vpt_synth_free.argtypes = [gridp]
    L.vpt_grid_from_nanovdb.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(gridp)]
    L.vpt_grid_read_nvdb.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(gridp)]
    L.vpt_grid_free.argtypes = [gridp]
    L.vpt_film_to_srgb8.argtypes = [fp, C.c_int64, C.c_int64, C.POINTER(C.c_uint8)]
    L.vpt_gpu_trace_jobs.argtypes = [vp, C.c_uint64, C.c_uint64, vp, vp, C.c_uint64, C.POINTER(C.c_uint64), vp]
    L.vpt_gpu_majorant_trace.argtypes = [vp, fp, fp, fp, C.c_int, C.POINTER(C.c_int)]
    L.vpt_dda_trace.argtypes = [C.POINTER(GridDesc), fp, fp, vp, C.c_int, C.POINTER(C.c_int)]
    L.vpt_gpu_set_rng_mode.argtypes = [vp, C.c_int]
    if hasattr(L, "vpt_gpu_set_pixel_chunk"):  # (A/B builds of older sources lack it; tests check the exports)
        L.vpt_gpu_set_pixel_chunk.argtypes = [vp, C.c_int]
    L.vpt_gpu_set_run_skipping.argtypes = [vp, C.c_int]
    L.vpt_gpu_kernel_variant.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    if hasattr(L, "vpt_gpu_set_film_order"):
        L.vpt_gpu_set_film_order.argtypes = [vp, C.c_int, C.c_uint64]
        L.vpt_gpu_film_order_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_uint64),
                                              C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.vpt_gpu_set_job_order.argtypes = [vp, C.c_int]
    L.vpt_gpu_set_job_order_tail.argtypes = [vp, C.c_int]
    L.vpt_gpu_tile_costs.argtypes = [vp, fp, C.POINTER(C.c_uint32)]
    L.vpt_gpu_set_tile_costs.argtypes = [vp, fp]
    L.vpt_gpu_set_job_permutation.argtypes = [vp, C.POINTER(C.c_uint32), C.c_uint64]
    if hasattr(L, "vpt_gpu_set_latency_kernel"):  # (A/B builds of older sources lack it; tests check the exports)
        L.vpt_gpu_set_latency_kernel.argtypes = [vp, C.c_int, C.c_int]
    if hasattr(L, "vpt_gpu_set_compaction"):
        L.vpt_gpu_set_compaction.argtypes = [vp, C.c_int]
        L.vpt_gpu_latency_kernel_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    if hasattr(L, "vpt_gpu_bind_thread_near"):
        L.vpt_gpu_bind_thread_near.argtypes = [vp, C.POINTER(C.c_int)]
    if hasattr(L, "vpt_gpu_stream_create"):
        L.vpt_gpu_stream_create.argtypes = [vp, C.POINTER(vp)]
        L.vpt_gpu_stream_destroy.argtypes = [vp, vp]
        L.vpt_gpu_stream_sync.argtypes = [vp, vp]
        L.vpt_gpu_film_alloc.argtypes = [vp, C.POINTER(vp)]
        L.vpt_gpu_film_free.argtypes = [vp, vp]
        L.vpt_gpu_film_flush_to_host.argtypes = [vp, vp, fp]
    if hasattr(L, "vpt_gpu_feed_open"):
        L.vpt_gpu_feed_open.argtypes = [vp, vp, vp, C.c_uint64, C.POINTER(vp)]
        L.vpt_gpu_feed_push.argtypes = [vp, C.POINTER(C.c_uint64), C.c_uint64]
        L.vpt_gpu_feed_close.argtypes = [vp]
        L.vpt_gpu_feed_query.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_uint64)]
        L.vpt_gpu_feed_destroy.argtypes = [vp]
    if hasattr(L, "vpt_gpu_feed_open_staged"):
        L.vpt_gpu_feed_open_staged.argtypes = [vp, vp, vp, C.c_uint64, C.POINTER(vp)]
        L.vpt_gpu_feed_collect.argtypes = [vp, fp]
    if hasattr(L, "vpt_gpu_feed_snapshot"):
        L.vpt_gpu_feed_snapshot.argtypes = [vp, fp]
        L.vpt_gpu_feed_backlog.argtypes = [vp, C.POINTER(C.c_uint64)]
        L.vpt_gpu_feed_prepare.argtypes = [vp, C.c_uint64, C.c_int]
    if hasattr(L, "vpt_gpu_feed_debug"):
        L.vpt_gpu_feed_debug.argtypes = [vp, C.c_int, C.POINTER(C.c_uint64)]
    if hasattr(L, "vpt_gpu_find_seeds"):
        L.vpt_gpu_find_seeds.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.c_int,
                                         C.POINTER(C.c_int)]
        L.vpt_gpu_setup_timings.argtypes = [vp, C.POINTER(C.c_double), C.c_int]
    _lib = L
    return L


def grid_from_nanovdb(buffer: bytes) -> "Grid":
    """vpt_grid_from_nanovdb: a NanoGrid<float> buffer flattened by the C++ reader (copied out)."""
    p = C.POINTER(GridDesc)()
    raw = C.create_string_buffer(bytes(buffer), len(buffer))
    check(lib().vpt_grid_from_nanovdb(raw, len(buffer), C.byref(p)), "vpt_grid_from_nanovdb")
    try:
        return Grid.from_desc(p.contents, copy=True)
    finally:
        lib().vpt_grid_free(p)


def read_nvdb_grid(path, name: str) -> "Grid | None":
    """vpt_grid_read_nvdb: the named float grid of a .nvdb file (C++ reader), or None if absent."""
    p = C.POINTER(GridDesc)()
    check(lib().vpt_grid_read_nvdb(str(path).encode(), name.encode(), C.byref(p)), "vpt_grid_read_nvdb")
    if not p:
        return None
    try:
        return Grid.from_desc(p.contents, copy=True)
    finally:
        lib().vpt_grid_free(p)


def check(rc: int, what: str = "") -> None:
    if rc != VPT_OK:
        msg = lib().vpt_last_error()
        raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
