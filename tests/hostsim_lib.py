"""ctypes binding of tests/native/libvpt_hostsim.so (the device state machine run on the CPU)."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

from volume_path_tracer_amd.capi import Configuration, Counters, GridDesc

NATIVE = Path(__file__).resolve().parent / "native"
LIB = NATIVE / "build" / "libvpt_hostsim.so"
_L = None


def lib():
    global _L
    if _L is None:
        subprocess.run(["make", "-s", "-C", str(NATIVE)], check=True)
        # hipcc links the host simulator against libamdhip64: torch's HIP runtime must be the process's
        # one (see volume_path_tracer_amd/capi.py lib())
        import torch  # noqa: F401
        L = C.CDLL(str(LIB))
        cfgp, gp, fp = C.POINTER(Configuration), C.POINTER(GridDesc), C.POINTER(C.c_float)
        L.vpths_render_jobs.argtypes = [cfgp, gp, gp, fp, C.c_uint64, C.c_uint64, fp, fp, C.POINTER(Counters)]
        L.vpths_fixed_leaf_max.argtypes = [gp, fp]
        L.vpths_render_jobs_mode.argtypes = [cfgp, gp, gp, fp, C.c_uint64, C.c_uint64, fp, fp, C.POINTER(Counters),
                                             C.c_int]
        L.vpths_render_jobs_order.argtypes = [cfgp, gp, gp, fp, C.c_uint64, C.c_uint64, fp, fp,
                                              C.POINTER(Counters), C.c_int, C.POINTER(C.c_uint32), C.c_int]
        L.vpths_probe.argtypes = [gp, C.POINTER(C.c_int32), C.c_int, fp, C.POINTER(C.c_int32), fp]
        L.vpths_check_runs.argtypes = [gp, C.POINTER(C.c_int64), C.POINTER(C.c_double)]
        L.vpths_check_runs.restype = C.c_int64
        L.vpths_check_walk.argtypes = [gp, C.POINTER(C.c_int64)]
        L.vpths_check_walk.restype = C.c_int64
        L.vpths_math_mismatches.argtypes = [C.c_int]
        L.vpths_math_mismatches.restype = C.c_int64
        L.vpths_pow2_mismatches.restype = C.c_int64
        L.vpths_walk_outside.argtypes = [C.c_int]
        L.vpths_walk_outside.restype = C.c_uint64
        _L = L
    return _L


def fptr(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_float))


def render_jobs(cfg, density, temperature, jid_begin, jid_count, records=False, bb=None, rng_mode=0, order=None,
                tail_waves=0):
    """order: tile ranks (uint32[T]) for a whole-wave range, taken in the GPU's job-order mapping
    (ordered_job) with the last tail_waves waves tile-major (-1: the same-tile order)."""
    film = np.zeros((cfg.height, cfg.width, 4), np.float32)
    tile_area = int(cfg.tile_size[0] * cfg.tile_size[1])
    rec = np.full((jid_count * tile_area, 3), np.nan, np.float32) if records else None
    cnt = Counters()
    op = None
    if order is not None:
        order = np.ascontiguousarray(order, np.uint32)
        op = order.ctypes.data_as(C.POINTER(C.c_uint32))
    rc = lib().vpths_render_jobs_order(C.byref(cfg), C.byref(density.desc),
                                       C.byref(temperature.desc) if temperature is not None else None,
                                       fptr(bb), jid_begin, jid_count, fptr(film), fptr(rec), C.byref(cnt), rng_mode,
                                       op, int(tail_waves))
    assert rc == 0
    return film, rec, cnt.as_dict()


def walk_outside(reset=True):
    """Walk-table lookups outside the padded table since the last reset (must stay 0)."""
    return int(lib().vpths_walk_outside(1 if reset else 0))


def fixed_leaf_max(grid):
    out = np.zeros(grid.leaf_count, np.float32)
    assert lib().vpths_fixed_leaf_max(C.byref(grid.desc), fptr(out)) == 0
    return out


def probe(grid, ijk):
    ijk = np.ascontiguousarray(ijk, np.int32).reshape(-1, 3)
    n = ijk.shape[0]
    val, maj = np.zeros(n, np.float32), np.zeros(n, np.float32)
    dim = np.zeros(n, np.int32)
    assert lib().vpths_probe(C.byref(grid.desc), ijk.ctypes.data_as(C.POINTER(C.c_int32)), n, fptr(val),
                             dim.ctypes.data_as(C.POINTER(C.c_int32)), fptr(maj)) == 0
    return val, dim, maj
