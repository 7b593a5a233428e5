"""Volume files -> flattened grids (the VolumeGrids::read_from_file seam, src/volume_grids.cpp:56-65).

A volume file holds a "density" grid and optionally a "temperature" grid.  Formats:

* ``.npz``  the flattened-grid arrays of ``vpt_grid_desc`` (``density/leaf_origin`` …), written by
            :func:`save_npz` — the interchange format for grids converted elsewhere;
* ``.nvdb`` NanoVDB files (see nvdb.py).

As in the reference, a file without a density grid is fatal (``nanovdb_read_grid_or_die``) and a
missing temperature grid only a warning.
"""
from __future__ import annotations

import sys
from pathlib import Path
from typing import Optional, Tuple

import numpy as np

from . import capi

_FIELDS = ("map_mat", "map_inv_mat", "map_vec", "background", "bbox_min", "bbox_max", "leaf_origin",
           "leaf_values", "leaf_max", "leaf_value_mask", "tile_origin", "tile_level", "tile_value",
           "tile_active", "lower_origin", "upper_origin")


def save_npz(path, density: capi.Grid, temperature: Optional[capi.Grid] = None) -> None:
    out = {}
    for name, g in (("density", density), ("temperature", temperature)):
        if g is None:
            continue
        d = g.desc
        out[f"{name}/map_mat"] = np.array(list(d.map_mat), np.float32)
        out[f"{name}/map_inv_mat"] = np.array(list(d.map_inv_mat), np.float32)
        out[f"{name}/map_vec"] = np.array(list(d.map_vec), np.float32)
        out[f"{name}/background"] = np.array([d.background], np.float32)
        out[f"{name}/bbox_min"] = np.array(list(d.index_bbox_min), np.int32)
        out[f"{name}/bbox_max"] = np.array(list(d.index_bbox_max), np.int32)
        for f in _FIELDS[6:]:
            a = getattr(g, f)
            if a is not None:
                out[f"{name}/{f}"] = a
    np.savez(path, **out)


def _grid_from_npz(z, name: str) -> Optional[capi.Grid]:
    keys = {k.split("/", 1)[1] for k in z.files if k.startswith(name + "/")}
    if not keys:
        return None
    kw = {f: z[f"{name}/{f}"] for f in _FIELDS if f in keys}
    kw["background"] = float(kw["background"][0])
    return capi.Grid(**kw)


def read_grids(path) -> Tuple[capi.Grid, Optional[capi.Grid]]:
    """(density, temperature-or-None) from a volume file; raises if there is no density grid."""
    path = Path(path)
    if not path.exists():
        raise FileNotFoundError(f"volume file {path} does not exist")
    if path.suffix == ".npz":
        with np.load(path, allow_pickle=False) as z:
            dens, temp = _grid_from_npz(z, "density"), _grid_from_npz(z, "temperature")
    elif path.suffix == ".nvdb":
        from . import nvdb

        grids = nvdb.read_grids(path, ("density", "temperature"))
        dens, temp = grids.get("density"), grids.get("temperature")
    else:
        raise ValueError(f"unsupported volume format {path.suffix!r} ({path})")
    if dens is None:
        raise ValueError(f"volume file {path} does not contain the \"density\" grid.")
    if temp is None:
        print(f"[vpt] warning: no \"temperature\" grid in {path}", file=sys.stderr)
    return dens, temp
