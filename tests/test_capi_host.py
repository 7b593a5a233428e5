"""Host-side checks of the C-ABI library (no GPU needed): exports, config reader, blackbody,
camera constants, TileProvider, and the loud failure when no HIP device is present."""
import ctypes as C
import json
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_lib as O
from volume_path_tracer_amd import capi
from volume_path_tracer_amd.render import TileProvider
from volume_path_tracer_amd.scenes import SCENE_DIR, parse_configuration, read_configuration, scene

ROOT = Path(__file__).resolve().parents[1]
G = ROOT / "tests" / "golden"


def declared_functions():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names |= set(re.findall(r"\b(vpt_[a-z0-9_]+)\s*\(", text))
    return names


def test_library_exports_every_declared_symbol():
    lib = capi.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", str(capi.LIB_PATH)], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (vpt_\w+)", out))
    declared = declared_functions()
    assert declared, "no declarations found"
    missing = declared - exported
    assert not missing, missing
    for n in declared:
        getattr(lib, n)  # resolvable through ctypes


def test_abi_version():
    assert capi.lib().vpt_abi_version() == 1


@pytest.mark.parametrize("name", ["wdas_cloud", "fire", "fire_lowscattering"])
def test_reference_scenes_parse(name):
    cfg = scene(name)
    raw = json.loads((SCENE_DIR / f"{name}.json").read_text())
    assert cfg.seed == raw["seed"] and cfg.num_waves == raw["num_waves"]
    assert [cfg.output_size[0], cfg.output_size[1]] == raw["output_size"]
    assert cfg.worker_parameters.max_depth == raw["worker_parameters"]["max_depth"]
    assert cfg.volume_path.decode() == raw["volume_path"]
    np.testing.assert_array_equal(np.float32(cfg.volume_parameters.sigma_s), np.float32(raw["volume_parameters"]["sigma_s"]))
    np.testing.assert_array_equal(np.asarray(cfg.camera_parameters.position, np.float32),
                                  np.asarray(raw["camera_parameters"]["position"], np.float32))


def _scene_text(mut=None):
    d = json.loads((SCENE_DIR / "wdas_cloud.json").read_text())
    if mut:
        mut(d)
    return json.dumps(d)


def test_config_missing_key_is_error():
    def drop(d):
        del d["worker_parameters"]["distant_light"]["multiplier"]
    with pytest.raises(RuntimeError, match="missing key"):
        parse_configuration(_scene_text(drop))


def test_config_unknown_key_is_error():
    def add(d):
        d["volume_parameters"]["density_scale"] = 2.0
    with pytest.raises(RuntimeError, match="unknown key"):
        parse_configuration(_scene_text(add))


def test_config_type_errors():
    for mut in (lambda d: d.__setitem__("seed", -1), lambda d: d.__setitem__("output_size", [1, 2, 3]),
                lambda d: d["worker_parameters"].__setitem__("use_jitter", 1)):
        with pytest.raises(RuntimeError):
            parse_configuration(_scene_text(mut))
    with pytest.raises(RuntimeError):
        parse_configuration("{")
    with pytest.raises(RuntimeError, match="cannot read"):
        read_configuration("/nonexistent/scene.json")


def test_blackbody_table_matches_oracle_and_kat():
    t = np.zeros((500, 3), np.float32)
    assert capi.lib().vpt_blackbody_table(t.ctypes.data_as(C.POINTER(C.c_float))) == 0
    np.testing.assert_array_equal(t, O.blackbody_table())
    kat = json.loads((G / "blackbody_kat.json").read_text())
    for c in kat["cases"]:
        out = np.zeros(3, np.float32)
        capi.lib().vpt_blackbody_xyz(t.ctypes.data_as(C.POINTER(C.c_float)), C.c_float(c["T"]),
                                     out.ctypes.data_as(C.POINTER(C.c_float)))
        np.testing.assert_array_equal(out, np.asarray(c["xyz"], np.float32))


def test_gpu_create_fails_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    from volume_path_tracer_amd.scenes import SynthGrid, workload
    wl = workload("c2", width=16, height=16, spp=1, grid_n=16)
    g = SynthGrid(0, 16)
    h = C.c_void_p()
    rc = capi.lib().vpt_gpu_create(C.byref(wl.cfg), C.byref(g.desc), None, None, 0, C.byref(h))
    assert rc == 2 and b"no HIP device" in capi.lib().vpt_last_error()


def test_grids_flatten_needs_no_device_and_create_from_fails_loudly_without_one():
    """vpt_grids_flatten is host work (run() overlaps it with the HIP runtime's start); the contexts made from its
    grids need a device, and say so without one."""
    import torch
    from volume_path_tracer_amd.scenes import SynthGrid, workload
    L = capi.lib()
    wl = workload("c4", width=16, height=16, spp=1, grid_n=32)
    d, t = SynthGrid(1, 32), SynthGrid(2, 32)
    g = C.c_void_p()
    assert L.vpt_grids_flatten(C.byref(d.desc), C.byref(t.desc), C.byref(g)) == 0 and g.value
    L.vpt_grids_free(g)
    assert L.vpt_grids_flatten(None, None, C.byref(g)) == 1  # VPT_E_INVALID
    g2 = C.c_void_p()
    assert L.vpt_grids_flatten(C.byref(d.desc), None, C.byref(g2)) == 0 and g2.value
    if not torch.cuda.is_available():
        devs = (C.c_int * 1)(0)
        outs = (C.c_void_p * 1)()
        rc = L.vpt_gpu_create_from(C.byref(wl.cfg), g2, None, devs, 1, outs)
        assert rc == 2 and b"no HIP device" in L.vpt_last_error() and not outs[0]
    L.vpt_grids_free(g2)
    L.vpt_grids_free(None)


def test_tile_provider_semantics():
    tp = TileProvider((20, 10), 3, (8, 8))
    assert tp.num_tiles == 3 * 2
    assert tp.job(0) == (0, 1) and tp.job(6) == (0, 2) and tp.job(13) == (1, 3)
    assert tp.compute_tile_rect(2) == (16, 0, 4, 8)   # clipped at the right edge
    assert tp.compute_tile_rect(5) == (16, 8, 4, 2)
    b, n = tp.next_batch(4)
    assert (b, n) == (0, 4) and tp.max_wave_idx == 1
    b, n = tp.next_batch(4)
    assert (b, n) == (4, 4) and tp.max_wave_idx == 2
    tp.stop_at_next_wave()
    b, n = tp.next_batch(100)
    assert (b, n) == (8, 4)  # finishes wave 2, never starts wave 3
    assert tp.next_batch(100)[1] == 0


def test_tuning_calls_reject_bad_arguments_without_a_device():
    """The scheduling knobs reject a null context before touching a device (their gate_idle 0 check is
    a GPU test: tests/test_gpu_production.py::test_latency_launch_knobs_keep_films_bit_exact)."""
    L = capi.lib()
    assert L.vpt_gpu_set_tuning(None, 6, 8, 0, 36, 4) != capi.VPT_OK
    assert b"null context" in L.vpt_last_error()
    assert L.vpt_gpu_set_latency_tuning(None, 0, 1, 65, 1, 1) != capi.VPT_OK
    assert b"null context" in L.vpt_last_error()


def test_grid_build_rejects_extents_beyond_the_24_bit_walk_index():
    """The device indexes the walk table with 24-bit multiplies: a lower-node extent whose x-y face
    reaches 2^24 cells is rejected at build time (VPT_E_INVALID) instead of diverging silently
    (ADVICE r02).  Two leaves 255 lower nodes apart in x and y: a 4100 x 4100-cell padded face."""
    vals = np.zeros((2, 512), np.float32)
    far = 255 * 128
    g = capi.Grid(map_mat=np.eye(3), map_inv_mat=np.eye(3), map_vec=[0, 0, 0], background=0.0,
                  bbox_min=[0, 0, 0], bbox_max=[far + 7, far + 7, 7],
                  leaf_origin=[[0, 0, 0], [far, far, 0]], leaf_values=vals, leaf_max=np.zeros(2, np.float32))
    out = np.zeros(2, np.float32)
    rc = capi.lib().vpt_fix_majorants(C.byref(g.desc), out.ctypes.data_as(C.POINTER(C.c_float)), 2)
    assert rc == 1, rc  # VPT_E_INVALID, before any table is allocated
    assert b"24-bit" in capi.lib().vpt_last_error()
