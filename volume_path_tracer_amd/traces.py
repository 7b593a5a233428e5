"""Debug traces in the reference's CSV formats.

* ``write_event_log`` -> ``log.csv`` of ``Logger<true>`` (src/worker.cpp:16-48): one line per
  event, ``name,values...`` (new_ray / scatter: origin xyz, direction xyz; sampled_point: point
  xyz, density; null / scatter_terminated / absorbed: the name only).
* ``write_majorant_trace`` -> ``majorant_trace.csv`` of ``Volume::log_majorant_trace``
  (src/volume.cpp:176-192): header ``X0,Y0,Z0,X1,Y1,Z1,T0,T1,Majorant`` and one row per segment.

Numbers are printed like ``std::ostream << float`` with the default precision (printf ``%g``),
the reference's ``print_csv`` (include/vpt/utils.hpp:16-24).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

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
