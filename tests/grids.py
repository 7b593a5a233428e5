"""Hand-built test grids that exercise every HDDA level: gaps between lower nodes (dim 128),
upper-node and root tiles (dim 128 / 4096), lower-node tiles (dim 8), negative coordinates."""
import numpy as np

from volume_path_tracer_amd import capi
from volume_path_tracer_amd.scenes import SynthGrid


def sparse_grid() -> capi.Grid:
    base = SynthGrid(1, 128).grid(copy=True)  # one lower node per copy
    offsets = np.array([[0, 0, 0], [256, 0, 0], [128, 128, 256], [-256, 128, 0], [0, -384, 128]], np.int32)
    origin = np.concatenate([base.leaf_origin + o for o in offsets])
    values = np.concatenate([base.leaf_values] * len(offsets))
    vmax = np.concatenate([base.leaf_max] * len(offsets))
    mask = np.concatenate([base.leaf_value_mask] * len(offsets))
    tiles = dict(
        # lower-node tiles inside the first copy's lower node, an upper-node tile in a gap, and an
        # active root tile far away on the +x side
        tile_origin=[[64, 0, 0], [64, 8, 0], [0, 72, 64], [128, 0, 0], [-128, -128, -128], [4096, 0, 0]],
        tile_level=[1, 1, 1, 2, 2, 3],
        tile_value=[0.3, 0.6, 0.05, 0.02, 0.1, 0.01],
        tile_active=[1, 1, 0, 1, 1, 1])
    lo = origin.min(0)
    hi = origin.max(0) + 7
    return capi.Grid(map_mat=list(base.desc.map_mat), map_inv_mat=list(base.desc.map_inv_mat),
                     map_vec=list(base.desc.map_vec), background=0.0, bbox_min=lo.tolist(), bbox_max=hi.tolist(),
                     leaf_origin=origin, leaf_values=values, leaf_max=vmax, leaf_value_mask=mask, **tiles)


def look_at(cfg, pos, look, up=(0.0, 1.0, 0.0)):
    cp = cfg.camera_parameters
    cp.position[:] = [float(v) for v in pos]
    cp.look[:] = [float(v) for v in look]
    cp.up[:] = [float(v) for v in up]


def tiles_only_grid() -> capi.Grid:
    """No leaves at all: an active upper-node tile, an active root tile and a lower-node tile
    (so every HDDA dim occurs and the leaf-slot table holds only tiles)."""
    return capi.Grid(map_mat=[1, 0, 0, 0, 1, 0, 0, 0, 1], map_inv_mat=[1, 0, 0, 0, 1, 0, 0, 0, 1],
                     map_vec=[-64.0, -64.0, -64.0], background=0.0, bbox_min=[0, 0, 0], bbox_max=[4095, 255, 255],
                     leaf_origin=np.zeros((0, 3), np.int32), leaf_values=np.zeros((0, 512), np.float32),
                     leaf_max=np.zeros(0, np.float32),
                     tile_origin=[[0, 0, 0], [128, 0, 0], [0, 128, 8], [4096, 0, 0]],
                     tile_level=[2, 2, 1, 3], tile_value=[0.02, 0.0, 0.5, 0.01], tile_active=[1, 0, 1, 1])


def signed_grid() -> capi.Grid:
    """The 64^3 cloud with the leaves of one slab negated (negative leaf maxima, so negative
    majorants deep in the slab and mixed signs at its faces), plus active lower-node tiles holding
    -0.3 and -0.0: majorants with the sign bit set, which the walk table must not take for its
    edge-cell flag (kWalkEdge)."""
    base = SynthGrid(1, 64).grid(copy=True)
    origin = base.leaf_origin.copy()
    values = base.leaf_values.copy()
    slab = origin[:, 0] < 32
    values[slab] = -values[slab]
    vmax = values.max(axis=1).astype(np.float32)
    tiles = dict(tile_origin=[[64, 0, 0], [64, 8, 0], [64, 16, 8]], tile_level=[1, 1, 1],
                 tile_value=[-0.3, -0.0, 0.2], tile_active=[1, 1, 1])
    lo = np.minimum(origin.min(0), 0)
    hi = np.maximum(origin.max(0) + 7, [71, 23, 15])
    return capi.Grid(map_mat=list(base.desc.map_mat), map_inv_mat=list(base.desc.map_inv_mat),
                     map_vec=list(base.desc.map_vec), background=0.0, bbox_min=lo.tolist(), bbox_max=hi.tolist(),
                     leaf_origin=origin, leaf_values=values, leaf_max=vmax, leaf_value_mask=base.leaf_value_mask,
                     **tiles)
