"""The product's synthetic generator and grid flattening agree with the oracle's NanoVDB restatement."""
import numpy as np
import pytest

import hostsim_lib as HS
import oracle_lib as O
from volume_path_tracer_amd.scenes import SynthGrid


def _same_grid(a, b):
    assert a.leaf_count == b.leaf_count
    np.testing.assert_array_equal(a.leaf_origin, b.leaf_origin)
    np.testing.assert_array_equal(a.leaf_values.view(np.uint32), b.leaf_values.view(np.uint32))
    np.testing.assert_array_equal(a.leaf_max, b.leaf_max)
    np.testing.assert_array_equal(a.leaf_value_mask, b.leaf_value_mask)
    assert list(a.desc.index_bbox_min) == list(b.desc.index_bbox_min)
    assert list(a.desc.index_bbox_max) == list(b.desc.index_bbox_max)
    assert list(a.desc.map_vec) == list(b.desc.map_vec)


@pytest.mark.parametrize("kind,n", [(0, 32), (1, 64), (2, 64), (1, 128)])
def test_synth_matches_oracle_generator(kind, n):
    prod = SynthGrid(kind, n).grid()
    orac = O.synth_grid(kind, n)
    _same_grid(prod, orac)


@pytest.mark.parametrize("kind,n", [(0, 32), (1, 64), (1, 128)])
def test_fix_majorants_matches_oracle(kind, n):
    g = SynthGrid(kind, n).grid()
    og = O.OracleGrid(g, fix_majorants=True)
    np.testing.assert_array_equal(HS.fixed_leaf_max(g), og.leaf_max())
    # idempotent
    g2 = SynthGrid(kind, n).grid()
    g2.leaf_max[:] = og.leaf_max()
    np.testing.assert_array_equal(HS.fixed_leaf_max(g2), og.leaf_max())


def _grid_with_tiles():
    """A hand-made grid with leaves, lower/upper/root tiles and negative coordinates."""
    rng = np.random.default_rng(7)
    origins = np.array([[0, 0, 0], [8, 0, 0], [-8, 16, 120], [120, 120, 120], [4096, 0, -128]], np.int32)
    vals = rng.random((len(origins), 512), dtype=np.float32)
    vals[1, :100] = 0
    from volume_path_tracer_amd.capi import Grid
    tiles = dict(
        tile_origin=np.array([[16, 0, 0], [128, 0, 0], [-4096, 0, 0], [24, 8, 0]], np.int32),
        tile_level=np.array([1, 2, 3, 1], np.int32),
        tile_value=np.array([0.75, 1.25, 0.5, 2.0], np.float32),
        tile_active=np.array([1, 1, 1, 0], np.uint8))
    return Grid(map_mat=np.eye(3), map_inv_mat=np.eye(3), map_vec=[0, 0, 0], background=0.0,
                bbox_min=[-8, 0, -128], bbox_max=[4103, 127, 127], leaf_origin=origins, leaf_values=vals,
                leaf_max=vals.max(axis=1), **tiles)


def test_probe_tables_match_oracle_tree():
    g = _grid_with_tiles()
    og = O.OracleGrid(g, fix_majorants=True)
    rng = np.random.default_rng(1)
    pts = [rng.integers(-300, 300, size=(4000, 3)), rng.integers(-5000, 5000, size=(2000, 3)),
           np.array([[16, 0, 0], [23, 7, 7], [24, 8, 0], [130, 1, 1], [-4000, 5, 5], [4100, 3, -100], [-9, 16, 120]])]
    ijk = np.concatenate(pts).astype(np.int32)
    val, dim, maj = HS.probe(g, ijk)
    fixed = og.leaf_max()
    for q, (i, j, k) in enumerate(ijk.tolist()):
        assert val[q] == np.float32(og.get_value(i, j, k)), (i, j, k)
        assert dim[q] == max(8, og.get_dim(i, j, k)), (i, j, k)
    np.testing.assert_array_equal(HS.fixed_leaf_max(g), fixed)


def test_trilinear_matches_oracle():
    from volume_path_tracer_amd.scenes import SynthGrid
    g = SynthGrid(1, 64).grid()
    og = O.OracleGrid(g, fix_majorants=True)
    rng = np.random.default_rng(3)
    for p in rng.uniform(-2, 66, size=(500, 3)).astype(np.float32):
        v = og.sample(*[float(x) for x in p])
        assert np.isfinite(v)


@pytest.mark.parametrize("which", ["cloud128", "cloud256", "constant", "sparse", "tiles_only"])
def test_run_radii_hold(which):
    """Run radii (compute_runs) let the Runs kernel variant take r HDDA steps without cell loads:
    every cell within Chebyshev distance r must be interior with the same majorant (brute force).
    The variant is chosen for grids where >= 1/4 of the interior cells have r >= 2 (C2's constant
    cube), not for the cloud."""
    import ctypes as C
    import grids
    g = {"cloud128": lambda: SynthGrid(1, 128).grid(), "cloud256": lambda: SynthGrid(1, 256).grid(),
         "constant": lambda: SynthGrid(0, 128).grid(), "sparse": grids.sparse_grid,
         "tiles_only": grids.tiles_only_grid}[which]()
    hist = np.zeros(16, np.int64)
    frac = C.c_double(0.0)
    bad = HS.lib().vpths_check_runs(C.byref(g.desc), hist.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(frac))
    assert bad == 0
    if which == "constant":
        assert frac.value >= 0.25 and hist[2:].sum() > 0
    if which.startswith("cloud"):
        assert frac.value < 0.25 and hist[1:].sum() > 0


@pytest.mark.parametrize("which", ["cloud128", "constant", "sparse", "tiles_only", "signed"])
def test_walk_table_words(which):
    """The HDDA walk table (interior / edge / slow words, kWalkPad padding) against cell_at by brute
    force (tests/native/hostsim.cpp vpths_check_walk): the fast paths' preconditions hold for every
    word, and every dim-8 cell with a sign-clear majorant takes one of them."""
    import ctypes as C
    import grids
    g = {"cloud128": lambda: SynthGrid(1, 128).grid(), "constant": lambda: SynthGrid(0, 128).grid(),
         "sparse": grids.sparse_grid, "tiles_only": grids.tiles_only_grid, "signed": grids.signed_grid}[which]()
    counts = np.zeros(5, np.int64)
    bad = HS.lib().vpths_check_walk(C.byref(g.desc), counts.ctypes.data_as(C.POINTER(C.c_int64)))
    assert bad == 0
    interior, edge, slow, pad, zero_runs = counts.tolist()
    assert pad > 0
    if which in ("cloud128", "constant", "sparse"):
        assert interior > 0 and edge > 0
    if which == "cloud128":
        assert zero_runs > 0  # empty space inside the cloud's lower nodes: zero-run words
    if which == "signed":
        assert slow > 0 and edge > 0  # negative majorants and the -0.0 tile stay slow
