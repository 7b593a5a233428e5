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


def mapped_grid(scale, angles_deg=(0.0, 0.0, 0.0), n=64, kind=1) -> capi.Grid:
    """The n^3 cloud (kind 1) or cube (kind 0) under a non-identity nanovdb::Map: index -> world =
    R(angles) @ diag(scale) @ ijk + vec, with vec putting the grid's centre at the world origin.  Both
    matrices are float32 roundings of the float64 ones, as NanoVDB stores mMatF / mInvMatF.  Voxel
    sizes far from 1 exercise the index-space lookahead and the walk-table padding argument
    (vpt_integrator.h walk_index)."""
    base = SynthGrid(kind, n).grid(copy=True)
    ax, ay, az = np.radians(angles_deg)
    rx = np.array([[1, 0, 0], [0, np.cos(ax), -np.sin(ax)], [0, np.sin(ax), np.cos(ax)]])
    ry = np.array([[np.cos(ay), 0, np.sin(ay)], [0, 1, 0], [-np.sin(ay), 0, np.cos(ay)]])
    rz = np.array([[np.cos(az), -np.sin(az), 0], [np.sin(az), np.cos(az), 0], [0, 0, 1]])
    m = rz @ ry @ rx @ np.diag(np.asarray(scale, np.float64))
    vec = -m @ np.full(3, n / 2.0)
    return capi.Grid(map_mat=m.astype(np.float32), map_inv_mat=np.linalg.inv(m).astype(np.float32),
                     map_vec=vec.astype(np.float32), background=0.0, bbox_min=list(base.desc.index_bbox_min),
                     bbox_max=list(base.desc.index_bbox_max), leaf_origin=base.leaf_origin, leaf_values=base.leaf_values,
                     leaf_max=base.leaf_max, leaf_value_mask=base.leaf_value_mask)


def mapped_scene(cfg, world_extent, sigma_scale):
    """Camera 2.6 world extents from the grid's centre (off axis), and sigma_a / sigma_s scaled so the
    optical depths match the unit-voxel scene (sigma is per world unit, volume.cpp:90-98 m_scale)."""
    look_at(cfg, (0.11 * world_extent, -0.07 * world_extent, -2.6 * world_extent), (0.0, 0.0, 0.0))
    v = cfg.volume_parameters
    v.sigma_a *= sigma_scale
    v.sigma_s *= sigma_scale


MAPPED_CASES = [  # (id, per-axis voxel size, rotation in degrees)
    ("small_voxels", (0.05, 0.04, 0.07), (20.0, -35.0, 10.0)),
    ("large_voxels", (20.0, 25.0, 18.0), (-15.0, 40.0, 5.0)),
    ("unit_rotated", (1.0, 1.0, 1.0), (30.0, 45.0, 60.0)),
]


def remapped(grid: capi.Grid, mat, vec) -> capi.Grid:
    """The same leaves under another index -> world map (mat, vec; float32 as NanoVDB stores them)."""
    m = np.asarray(mat, np.float64)
    return capi.Grid(map_mat=m.astype(np.float32), map_inv_mat=np.linalg.inv(m).astype(np.float32),
                     map_vec=np.asarray(vec, np.float32), background=float(grid.desc.background),
                     bbox_min=list(grid.desc.index_bbox_min), bbox_max=list(grid.desc.index_bbox_max),
                     leaf_origin=grid.leaf_origin, leaf_values=grid.leaf_values, leaf_max=grid.leaf_max,
                     leaf_value_mask=grid.leaf_value_mask)


def temperature_pair(kind):
    """(density, temperature) grids for the temperature sampler: "same" = the fire stand-in (one topology, one map); "shifted" = the temperature
    grid moved by (3, -5, 2) world units (its corners fall in other 8^3 cells for part of the
    lookups, and the joint values at the density leaves come from its tiles and background too);
    "half_voxels" = a 128^3 temperature grid of 0.5-unit voxels over the 64^3 density (mostly the
    temperature grid's own lookups); "sparse" = the sparse grid of every HDDA level, moved as in
    "shifted", as temperature over the 128^3 cloud (its lower-node tiles inside the density leaves)."""
    if kind == "sparse":
        t = sparse_grid()
        return SynthGrid(1, 128).grid(copy=True), remapped(t, np.eye(3), np.asarray(t.desc.map_vec, np.float64) + (3.0, -5.0, 2.0))
    dens = SynthGrid(1, 64).grid(copy=True)
    if kind == "same":
        return dens, SynthGrid(2, 64).grid(copy=True)
    if kind == "shifted":
        t = SynthGrid(2, 64).grid(copy=True)
        return dens, remapped(t, np.eye(3), np.asarray(t.desc.map_vec, np.float64) + (3.0, -5.0, 2.0))
    if kind == "half_voxels":
        return dens, remapped(SynthGrid(2, 128).grid(copy=True), 0.5 * np.eye(3), (0.0, 0.0, 0.0))
    raise ValueError(kind)

