"""Debug traces in the reference's CSV formats.

* ``write_event_log`` -> ``log.csv`` of ``Logger<true>`` (src/worker.cpp:16-48): one line per
  event, ``name,values...`` (new_ray / scatter: origin xyz, direction xyz; sampled_point: point
  xyz, density; null / scatter_terminated / absorbed: the name only).
* ``write_majorant_trace`` -> ``majorant_trace.csv`` of ``Volume::log_majorant_trace``
  (src/volume.cpp:176-192): header ``X0,Y0,Z0,X1,Y1,Z1,T0,T1,Majorant`` and one row per segment.
* ``dda_trace`` / ``write_dda_trace`` -> ``dda_trace.csv`` of ``Volume::log_dda_trace``
  (src/volume.cpp:194-225): header ``X,Y,Z,T,Value,Dim_getdim,Dim_nodeinfo,Active,Maximum`` and one
  row per voxel of the unit DDA (computed by the library's ``vpt_dda_trace`` on the host).

Numbers are printed like ``std::ostream << float`` with the default precision (printf ``%g``),
the reference's ``print_csv`` (include/vpt/utils.hpp:16-24).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

import ctypes as C

from . import capi
from .capi import EVENT_NAMES

_NVALS = {0: 6, 1: 4, 2: 0, 3: 0, 4: 6, 5: 0}


def fmt(x) -> str:
    """std::ostream << (float)x with default flags: %g, 6 significant digits."""
    return "%g" % float(np.float32(x))


def event_lines(events) -> list:
    out = []
    for e in events:
        t = int(e["type"])
        vals = [fmt(v) for v in e["v"][: _NVALS[t]]]
        out.append(",".join([EVENT_NAMES[t]] + vals))
    return out


def write_event_log(events, path="log.csv") -> None:
    Path(path).write_text("".join(line + "\n" for line in event_lines(events)))


def majorant_lines(rows) -> list:
    out = ["X0,Y0,Z0,X1,Y1,Z1,T0,T1,Majorant"]
    out += [",".join(fmt(v) for v in r) for r in np.asarray(rows, np.float32).reshape(-1, 9)]
    return out


def write_majorant_trace(rows, path="majorant_trace.csv") -> None:
    Path(path).write_text("".join(line + "\n" for line in majorant_lines(rows)))


def dda_trace(grid: "capi.Grid", origin, direction, max_rows: int = 1 << 20):
    """Volume::log_dda_trace rows (capi.DDA_ROW_DTYPE) for one world ray, or None when the ray
    misses the index bbox (the reference then writes no file)."""
    o = np.ascontiguousarray(origin, np.float32)
    d = np.ascontiguousarray(direction, np.float32)
    rows = np.zeros(max_rows, capi.DDA_ROW_DTYPE)
    n = C.c_int(0)
    fp = C.POINTER(C.c_float)
    capi.check(capi.lib().vpt_dda_trace(C.byref(grid.desc), o.ctypes.data_as(fp), d.ctypes.data_as(fp),
                                        rows.ctypes.data_as(C.c_void_p), max_rows, C.byref(n)), "vpt_dda_trace")
    if n.value < 0:
        return None
    if n.value > max_rows:
        raise RuntimeError(f"dda_trace: {n.value} voxels exceed max_rows {max_rows}")
    return rows[: n.value].copy()


def dda_lines(rows) -> list:
    out = ["X,Y,Z,T,Value,Dim_getdim,Dim_nodeinfo,Active,Maximum"]
    for r in rows:
        i, j, k = (int(v) for v in r["ijk"])
        out.append(",".join([str(i), str(j), str(k), fmt(r["t"]), fmt(r["value"]), str(int(r["dim_getdim"])),
                             str(int(r["dim_nodeinfo"])), str(int(r["active"])), fmt(r["maximum"])]))
    return out


def write_dda_trace(rows, path="dda_trace.csv") -> None:
    """No file for a ray that misses (rows is None), like the reference."""
    if rows is None:
        return
    Path(path).write_text("".join(line + "\n" for line in dda_lines(rows)))
