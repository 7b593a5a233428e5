"""NanoVDB ``.nvdb`` files <-> flattened grids (``vpt_grid_desc``), SURVEY §8f.

The reference loads its volumes with ``nanovdb::io::readGrid(path, "density" | "temperature")``
(src/volume_grids.cpp:38-65).  NanoVDB (openvdb submodule, pinned by the reference's
external/CMakeLists.txt but not vendored in /root/reference) is not available here, so this module
restates its published on-disk layout (NanoVDB 32.x, float grids, ``NANOVDB_USE_SINGLE_ROOT_KEY``):

  file     := segment*;  segment := FileHeader, gridCount x (FileMetaData, name), gridCount x blob
  FileHeader   16 B: magic u64 ("NanoVDB0"/"NanoVDB2"), version u32, gridCount u16, codec u16
  FileMetaData 176 B: gridSize, fileSize, nameKey, voxelCount (u64), gridType u32, gridClass u32,
               worldBBox 6xf64, indexBBox 6xi32, voxelSize 3xf64, nameSize u32 (incl. NUL),
               nodeCount 4xu32, tileCount 3xu32, codec u16, pad u16, version u32
  blob         codec NONE: the grid buffer (gridSize bytes); ZIP: u64 n + zlib stream of n bytes
  grid buffer  GridData (672 B: map floats at 296) | TreeData (64 B: node byte offsets [leaf, lower,
               upper, root] from TreeData) | RootData (64 B: bbox, tableSize, background, stats) +
               tiles (32 B: key u64, child i64 byte offset from RootData, state u32, value f32) |
               upper nodes (InternalData<.,5>: bbox, flags, value/child masks 4096 B each, stats,
               table of 32768 x 8 B at 8256) | lower nodes (InternalData<.,4>: masks 512 B,
               table of 4096 x 8 B at 1088) | leaves (2144 B: bboxMin, bboxDif, flags, value mask
               64 B at 16, min/max/avg/std at 80, values at 96)

Parity unpinned: no .nvdb file ships with the reference (volumes/ is absent), so the reader is
checked only against ``write_nvdb`` round trips and the grids' own semantics (tests/test_image_io.py: test_nvdb_roundtrip, test_nvdb_rejects_garbage).
"""
from __future__ import annotations

import struct
import zlib
from pathlib import Path
from typing import Dict, Iterable, Optional

import numpy as np

from . import capi

MAGIC_NUMBER = 0x304244566F6E614E  # "NanoVDB0"
MAGIC_GRID = 0x314244566F6E614E    # "NanoVDB1"
MAGIC_FILE = 0x324244566F6E614E    # "NanoVDB2"
VERSION = (32 << 21) | (7 << 10) | 0
GRID_TYPE_FLOAT = 1
GRID_CLASS_FOG = 2
CODEC_NONE, CODEC_ZIP = 0, 1

GRID_DATA_SIZE, TREE_DATA_SIZE, ROOT_DATA_SIZE, ROOT_TILE_SIZE = 672, 64, 64, 32
UPPER_TABLE, UPPER_SIZE = 8256, 8256 + 32768 * 8
LOWER_TABLE, LOWER_SIZE = 1088, 1088 + 4096 * 8
LEAF_VALUES, LEAF_SIZE = 96, 96 + 512 * 4
_META = struct.Struct("<4Q2I6d6i3dI4I3IHHI")
assert _META.size == 176


class NvdbError(ValueError):
    pass


# ---------------------------------------------------------------------------------------------
# reading


def _segments(data: bytes):
    """Yield (name, gridType, codec, blob bytes) for every grid in the file."""
    pos = 0
    while pos + 16 <= len(data):
        magic, version, count, codec = struct.unpack_from("<QIHH", data, pos)
        if magic not in (MAGIC_NUMBER, MAGIC_FILE):
            if pos == 0:
                raise NvdbError("not a NanoVDB file (bad magic)")
            break
        if (version >> 21) != 32:
            raise NvdbError(f"unsupported NanoVDB major version {version >> 21}")
        pos += 16
        metas = []
        for _ in range(count):
            m = _META.unpack_from(data, pos)
            pos += _META.size
            name_size = m[21]
            name = data[pos:pos + name_size].split(b"\0", 1)[0].decode()
            pos += name_size
            metas.append((name, m[0], m[4], m[-3]))
        for name, grid_size, gtype, gcodec in metas:
            c = gcodec
            if c == CODEC_NONE:
                blob = data[pos:pos + grid_size]
                pos += grid_size
            elif c == CODEC_ZIP:
                (n,) = struct.unpack_from("<Q", data, pos)
                blob = zlib.decompress(data[pos + 8:pos + 8 + n])
                pos += 8 + n
            else:
                raise NvdbError(f"grid {name!r}: codec {c} (BLOSC) is not supported")
            if len(blob) != grid_size:
                raise NvdbError(f"grid {name!r}: truncated buffer")
            yield name, gtype, blob


def _mask_bits(buf: np.ndarray, off: int, nbits: int) -> np.ndarray:
    words = buf[off:off + nbits // 8].view("<u8")
    return np.unpackbits(words.view(np.uint8), bitorder="little").astype(bool)


def grid_from_buffer(blob: bytes) -> capi.Grid:
    """One NanoGrid<float> buffer -> capi.Grid (leaves, tiles and node lists)."""
    buf = np.frombuffer(blob, np.uint8)
    magic, = struct.unpack_from("<Q", blob, 0)
    if magic not in (MAGIC_NUMBER, MAGIC_GRID):
        raise NvdbError("grid buffer: bad magic")
    version, = struct.unpack_from("<I", blob, 16)  # GridData::mVersion
    if (version >> 21) != 32:
        raise NvdbError(f"grid buffer: unsupported NanoVDB major version {version >> 21}")
    gtype, = struct.unpack_from("<I", blob, 636)
    if gtype != GRID_TYPE_FLOAT:
        raise NvdbError(f"grid buffer: grid type {gtype} is not float")
    mat = np.frombuffer(blob, "<f4", 9, 296)
    inv = np.frombuffer(blob, "<f4", 9, 296 + 36)
    vec = np.frombuffer(blob, "<f4", 3, 296 + 72)
    tree = GRID_DATA_SIZE
    node_off = struct.unpack_from("<4q", blob, tree)
    root = tree + node_off[3]
    bbox = struct.unpack_from("<6i", blob, root)
    table_size, background = struct.unpack_from("<If", blob, root + 24)

    leaf_origin, leaf_at, tiles, lowers, uppers = [], [], [], [], []
    for t in range(table_size):
        p = root + ROOT_DATA_SIZE + t * ROOT_TILE_SIZE
        key, child, state, value = struct.unpack_from("<QqIf", blob, p)
        o = [(((key >> s) & ((1 << 21) - 1)) << 12) & 0xFFFFFFFF for s in (42, 21, 0)]
        o = [v - (1 << 32) if v >= (1 << 31) else v for v in o]
        if child == 0:
            tiles.append((o, 3, value, state))
            continue
        up = root + child
        uppers.append(o)
        ucm = _mask_bits(buf, up + 32 + 4096, 32768)
        uvm = _mask_bits(buf, up + 32, 32768)
        utab = buf[up + UPPER_TABLE:up + UPPER_SIZE]
        for n in np.nonzero(~ucm & (uvm | (utab.view("<f4")[0::2] != np.float32(background))))[0]:
            i, j, k = n >> 10, (n >> 5) & 31, n & 31
            tiles.append(([o[0] + (i << 7), o[1] + (j << 7), o[2] + (k << 7)], 2,
                          float(utab.view("<f4")[2 * n]), int(uvm[n])))
        uchild = utab.view("<i8")
        for n in np.nonzero(ucm)[0]:
            lo = up + int(uchild[n])
            lorg = [o[0] + ((n >> 10) << 7), o[1] + (((n >> 5) & 31) << 7), o[2] + ((n & 31) << 7)]
            lowers.append(lorg)
            lcm = _mask_bits(buf, lo + 32 + 512, 4096)
            lvm = _mask_bits(buf, lo + 32, 4096)
            ltab = buf[lo + LOWER_TABLE:lo + LOWER_SIZE]
            lval = ltab.view("<f4")[0::2]
            sel = np.nonzero(~lcm & (lvm | (lval != np.float32(background))))[0]
            for n2 in sel:
                tiles.append(([lorg[0] + ((n2 >> 8) << 3), lorg[1] + (((n2 >> 4) & 15) << 3),
                               lorg[2] + ((n2 & 15) << 3)], 1, float(lval[n2]), int(lvm[n2])))
            lchild = ltab.view("<i8")
            ch = np.nonzero(lcm)[0]
            if ch.size:
                leaf_at.append(lo + lchild[ch])
                leaf_origin.append(np.stack([lorg[0] + ((ch >> 8) << 3), lorg[1] + (((ch >> 4) & 15) << 3),
                                             lorg[2] + ((ch & 15) << 3)], axis=1))
    if leaf_at:
        at = np.concatenate(leaf_at)
        origin = np.concatenate(leaf_origin).astype(np.int32)
    else:
        at, origin = np.zeros(0, np.int64), np.zeros((0, 3), np.int32)
    n = at.size
    # leaves are one contiguous array (TreeData node offset 0): index them by their byte offset
    base = tree + node_off[0]
    rel = at.astype(np.int64) - base
    if n and (np.any(rel < 0) or np.any(rel % LEAF_SIZE) or np.any(rel // LEAF_SIZE >= (len(blob) - base) // LEAF_SIZE)):
        raise NvdbError("grid buffer: leaf pointer outside the leaf array")
    count = (len(blob) - base) // LEAF_SIZE if n else 0
    arr = buf[base:base + count * LEAF_SIZE].reshape(count, LEAF_SIZE) if n else np.zeros((0, LEAF_SIZE), np.uint8)
    raw = arr[rel // LEAF_SIZE] if n else arr
    values = np.ascontiguousarray(raw[:, LEAF_VALUES:]).view("<f4").reshape(n, 512)
    masks = np.ascontiguousarray(raw[:, 16:80]).view("<u8").reshape(n, 8)
    leaf_max = np.ascontiguousarray(raw[:, 84:88]).view("<f4").reshape(n)
    kw = {}
    if tiles:
        kw = dict(tile_origin=np.array([t[0] for t in tiles], np.int32),
                  tile_level=np.array([t[1] for t in tiles], np.int32),
                  tile_value=np.array([t[2] for t in tiles], np.float32),
                  tile_active=np.array([1 if t[3] else 0 for t in tiles], np.uint8))
    return capi.Grid(map_mat=mat, map_inv_mat=inv, map_vec=vec, background=background,
                     bbox_min=bbox[:3], bbox_max=bbox[3:], leaf_origin=origin, leaf_values=values,
                     leaf_max=leaf_max, leaf_value_mask=masks,
                     lower_origin=np.array(lowers, np.int32).reshape(-1, 3) if lowers else None,
                     upper_origin=np.array(uppers, np.int32).reshape(-1, 3) if uppers else None, **kw)


def read_grids(path, names: Iterable[str] = ("density", "temperature")) -> Dict[str, capi.Grid]:
    """The named float grids of a .nvdb file (missing names are absent from the result)."""
    want = set(names)
    out: Dict[str, capi.Grid] = {}
    for name, gtype, blob in _segments(Path(path).read_bytes()):
        if name in want and name not in out:
            if gtype != GRID_TYPE_FLOAT:
                raise NvdbError(f"grid {name!r} is not a float grid (type {gtype})")
            out[name] = grid_from_buffer(blob)
    return out


# ---------------------------------------------------------------------------------------------
# writing (tests and tools: converting flattened grids to .nvdb)


def _key(o) -> int:
    m = (1 << 21) - 1
    u = [(int(v) & 0xFFFFFFFF) >> 12 for v in o]
    return (u[2] & m) | ((u[1] & m) << 21) | ((u[0] & m) << 42)


def _stats(v: np.ndarray):
    if v.size == 0:
        return 0.0, 0.0, 0.0, 0.0
    v64 = v.astype(np.float64)
    return float(v.min()), float(v.max()), float(v64.mean()), float(v64.std())


def buffer_from_grid(g: capi.Grid, name: str) -> bytes:
    """capi.Grid -> NanoGrid<float> buffer (breadth-first node order, as the NanoVDB builder)."""
    d = g.desc
    bg = np.float32(d.background)
    n = g.leaf_count
    lo_of_leaf = {}
    for li in range(n):
        o = tuple(int(v) for v in g.leaf_origin[li])
        lo_of_leaf.setdefault((o[0] & ~127, o[1] & ~127, o[2] & ~127), []).append(li)
    t1, t2, t3 = {}, {}, {}
    if g.tile_origin is not None:
        for o, lvl, val, act in zip(g.tile_origin, g.tile_level, g.tile_value, g.tile_active):
            o = tuple(int(v) for v in o)
            {1: t1, 2: t2, 3: t3}[int(lvl)][o] = (np.float32(val), int(act))
    lowers = set(lo_of_leaf)
    lowers |= {(o[0] & ~127, o[1] & ~127, o[2] & ~127) for o in t1}
    if g.lower_origin is not None:
        lowers |= {tuple(int(v) & ~127 for v in o) for o in g.lower_origin}
    uppers = {(o[0] & ~4095, o[1] & ~4095, o[2] & ~4095) for o in lowers}
    uppers |= {(o[0] & ~4095, o[1] & ~4095, o[2] & ~4095) for o in t2}
    if g.upper_origin is not None:
        uppers |= {tuple(int(v) & ~4095 for v in o) for o in g.upper_origin}
    uppers = sorted(uppers)
    lowers = sorted(lowers)
    root_tiles = [(o, t3[o]) for o in sorted(t3) if o not in set(uppers)]
    leaf_order = [li for lo in lowers for li in sorted(lo_of_leaf.get(lo, []),
                                                        key=lambda i: tuple(g.leaf_origin[i]))]
    table_size = len(uppers) + len(root_tiles)
    root_bytes = ROOT_DATA_SIZE + table_size * ROOT_TILE_SIZE
    off_root = GRID_DATA_SIZE + TREE_DATA_SIZE
    off_upper = off_root + root_bytes
    off_lower = off_upper + len(uppers) * UPPER_SIZE
    off_leaf = off_lower + len(lowers) * LOWER_SIZE
    total = off_leaf + len(leaf_order) * LEAF_SIZE
    buf = bytearray(total)
    upper_pos = {o: off_upper + i * UPPER_SIZE for i, o in enumerate(uppers)}
    lower_pos = {o: off_lower + i * LOWER_SIZE for i, o in enumerate(lowers)}
    leaf_pos = {li: off_leaf + i * LEAF_SIZE for i, li in enumerate(leaf_order)}

    all_vals = [g.leaf_values.reshape(-1)] if n else []
    # leaves, all at once (in leaf_order): the active voxels' bbox, the value mask, min / stored max / mean /
    # std of the 512 values, the values
    if leaf_order:
        order = np.asarray(leaf_order, np.int64)
        lv = np.asarray(g.leaf_values).reshape(n, 512)[order]
        lm = np.ascontiguousarray(np.asarray(g.leaf_value_mask).reshape(n, 8)[order], "<u8")
        bits = np.unpackbits(lm.view(np.uint8).reshape(-1, 64), axis=1, bitorder="little").astype(bool).reshape(-1, 8, 8, 8)
        lo_b, dif_b = [], []
        for ax in ((2, 3), (1, 3), (1, 2)):  # bit n = x << 6 | y << 3 | z
            a = bits.any(axis=ax)
            has = a.any(1)
            first = np.where(has, a.argmax(1), 0)
            last = np.where(has, 7 - a[:, ::-1].argmax(1), 0)
            lo_b.append(first)
            dif_b.append(last - first)
        rec = np.zeros(len(order), np.dtype([("bmin", "<i4", 3), ("bdif", "u1", 3), ("flags", "u1"), ("mask", "<u8", 8),
                                              ("stats", "<f4", 4), ("vals", "<f4", 512)]))
        assert rec.dtype.itemsize == LEAF_SIZE
        rec["bmin"] = np.asarray(g.leaf_origin).reshape(n, 3)[order].astype(np.int64) + np.stack(lo_b, 1)
        rec["bdif"] = np.stack(dif_b, 1)
        rec["mask"] = lm
        v64 = lv.astype(np.float64)
        rec["stats"][:, 0] = lv.min(1)
        rec["stats"][:, 1] = np.asarray(g.leaf_max).reshape(n)[order]
        rec["stats"][:, 2] = v64.mean(1)
        rec["stats"][:, 3] = v64.std(1)
        rec["vals"] = lv
        buf[off_leaf:off_leaf + len(order) * LEAF_SIZE] = rec.tobytes()
    # lower nodes
    for lo, p in lower_pos.items():
        tab = np.zeros(4096, "<i8")
        tabf = tab.view("<f4")
        tabf[0::2] = bg
        vm = np.zeros(4096, bool)
        cm = np.zeros(4096, bool)
        for li in lo_of_leaf.get(lo, []):
            o = g.leaf_origin[li]
            s = (((int(o[0]) & 127) >> 3) << 8) | (((int(o[1]) & 127) >> 3) << 4) | ((int(o[2]) & 127) >> 3)
            cm[s] = True
            tab[s] = leaf_pos[li] - p
        for o, (val, act) in t1.items():
            if (o[0] & ~127, o[1] & ~127, o[2] & ~127) != lo:
                continue
            s = (((o[0] & 127) >> 3) << 8) | (((o[1] & 127) >> 3) << 4) | ((o[2] & 127) >> 3)
            if cm[s]:
                continue
            tabf[2 * s] = val
            vm[s] = bool(act)
        struct.pack_into("<6i", buf, p, *lo, *(c + 127 for c in lo))
        buf[p + 32:p + 544] = np.packbits(vm, bitorder="little").tobytes()
        buf[p + 544:p + 1056] = np.packbits(cm, bitorder="little").tobytes()
        buf[p + LOWER_TABLE:p + LOWER_SIZE] = tab.tobytes()
    # upper nodes
    for up, p in upper_pos.items():
        tab = np.zeros(32768, "<i8")
        tabf = tab.view("<f4")
        tabf[0::2] = bg
        vm = np.zeros(32768, bool)
        cm = np.zeros(32768, bool)
        for lo in lowers:
            if (lo[0] & ~4095, lo[1] & ~4095, lo[2] & ~4095) != up:
                continue
            s = (((lo[0] & 4095) >> 7) << 10) | (((lo[1] & 4095) >> 7) << 5) | ((lo[2] & 4095) >> 7)
            cm[s] = True
            tab[s] = lower_pos[lo] - p
        for o, (val, act) in t2.items():
            if (o[0] & ~4095, o[1] & ~4095, o[2] & ~4095) != up:
                continue
            s = (((o[0] & 4095) >> 7) << 10) | (((o[1] & 4095) >> 7) << 5) | ((o[2] & 4095) >> 7)
            if cm[s]:
                continue
            tabf[2 * s] = val
            vm[s] = bool(act)
        struct.pack_into("<6i", buf, p, *up, *(c + 4095 for c in up))
        buf[p + 32:p + 4128] = np.packbits(vm, bitorder="little").tobytes()
        buf[p + 4128:p + 8224] = np.packbits(cm, bitorder="little").tobytes()
        buf[p + UPPER_TABLE:p + UPPER_SIZE] = tab.tobytes()
    # root
    mn, mx, avg, std = _stats(np.concatenate(all_vals)) if all_vals else (0.0, 0.0, 0.0, 0.0)
    struct.pack_into("<6iIf4f", buf, off_root, *d.index_bbox_min, *d.index_bbox_max, table_size, float(bg),
                     mn, mx, avg, std)
    entries = [(_key(o), upper_pos[o] - off_root, 0, float(bg)) for o in uppers]
    entries += [(_key(o), 0, int(act), float(val)) for o, (val, act) in root_tiles]
    for t, (key, child, state, value) in enumerate(sorted(entries)):
        struct.pack_into("<QqIf", buf, off_root + ROOT_DATA_SIZE + t * ROOT_TILE_SIZE, key, child, state, value)
    # tree
    struct.pack_into("<4q3I3IQ", buf, GRID_DATA_SIZE,
                     (off_leaf - GRID_DATA_SIZE) if leaf_order else 0,
                     (off_lower - GRID_DATA_SIZE) if lowers else 0,
                     (off_upper - GRID_DATA_SIZE) if uppers else 0,
                     off_root - GRID_DATA_SIZE,
                     len(leaf_order), len(lowers), len(uppers),
                     len(t1), len(t2), len(root_tiles), int(sum(int(m).bit_count() for m in g.leaf_value_mask.reshape(-1))))
    # grid
    nm = name.encode()[:255]
    struct.pack_into("<QQIIIIQ", buf, 0, MAGIC_GRID, 0xFFFFFFFFFFFFFFFF, VERSION, 0, 0, 1, total)
    buf[40:40 + len(nm)] = nm
    struct.pack_into("<9f9f3ff", buf, 296, *d.map_mat, *d.map_inv_mat, *d.map_vec, 1.0)
    md = np.array(list(d.map_mat), np.float64)
    mi = np.array(list(d.map_inv_mat), np.float64)
    struct.pack_into("<9d9d3dd", buf, 296 + 88, *md, *mi, *np.array(list(d.map_vec), np.float64), 1.0)
    struct.pack_into("<3d", buf, 608, float(d.map_mat[0]), float(d.map_mat[4]), float(d.map_mat[8]))
    struct.pack_into("<IIqII", buf, 632, GRID_CLASS_FOG, GRID_TYPE_FLOAT, 0, 0, 0)
    return bytes(buf)


def write_nvdb(path, grids: Dict[str, Optional[capi.Grid]], codec: int = CODEC_NONE) -> None:
    """Write float grids as one NanoVDB segment (codec NONE or ZIP)."""
    items = [(k, g) for k, g in grids.items() if g is not None]
    blobs = [buffer_from_grid(g, k) for k, g in items]
    out = bytearray(struct.pack("<QIHH", MAGIC_FILE, VERSION, len(items), codec))
    payload = []
    for (name, g), blob in zip(items, blobs):
        d = g.desc
        nb = name.encode() + b"\0"
        enc = blob if codec == CODEC_NONE else zlib.compress(blob)
        body = enc if codec == CODEC_NONE else struct.pack("<Q", len(enc)) + enc
        payload.append(body)
        out += _META.pack(len(blob), len(body), 0, int(sum(int(m).bit_count() for m in g.leaf_value_mask.reshape(-1))),
                          GRID_TYPE_FLOAT, GRID_CLASS_FOG, 0, 0, 0, 0, 0, 0,
                          *d.index_bbox_min, *d.index_bbox_max, 1.0, 1.0, 1.0, len(nb),
                          g.leaf_count, 0, 0, 0, 0, 0, 0, codec, 0, VERSION)
        out += nb
    for body in payload:
        out += body
    Path(path).write_bytes(bytes(out))
