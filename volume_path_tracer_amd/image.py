"""Output image: film -> 8-bit sRGB -> PNG (the headless half of src/main.cpp).

``film_to_image`` is the C-ABI ``vpt_film_to_srgb8`` (film_to_image, src/main.cpp:12-24, with the
xyz_to_linsrgb / linsrgb_to_srgb of include/vpt/color.hpp:8-30).  ``save_png`` writes what
``Image<unsigned char,3>::save`` writes (src/image_io.cpp:18-58: 8-bit truecolor, no alpha, rows
top to bottom); the pixel bytes are identical, the deflate stream is zlib's rather than spng's.
"""
from __future__ import annotations

import ctypes as C
import struct
import zlib
from pathlib import Path

import numpy as np

from . import capi


def film_to_image(film: np.ndarray) -> np.ndarray:
    """float32 [H][W][4] XYZW film -> uint8 [H][W][3] sRGB image."""
    film = np.ascontiguousarray(film, dtype=np.float32)
    if film.ndim != 3 or film.shape[2] != 4:
        raise ValueError(f"film must be [H][W][4], got {film.shape}")
    h, w = film.shape[:2]
    out = np.empty((h, w, 3), dtype=np.uint8)
    L = capi.lib()
    capi.check(L.vpt_film_to_srgb8(film.ctypes.data_as(C.POINTER(C.c_float)), w, h,
                                   out.ctypes.data_as(C.POINTER(C.c_uint8))), "vpt_film_to_srgb8")
    return out


def _chunk(tag: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def encode_png(rgb: np.ndarray) -> bytes:
    """uint8 [H][W][3] (or uint16) -> PNG bytes (truecolor, filter 0 per row)."""
    rgb = np.ascontiguousarray(rgb)
    if rgb.ndim != 3 or rgb.shape[2] != 3 or rgb.dtype not in (np.uint8, np.uint16):
        raise ValueError("encode_png wants uint8/uint16 [H][W][3]")
    h, w = rgb.shape[:2]
    depth = 8 * rgb.dtype.itemsize
    rows = rgb.astype(rgb.dtype.newbyteorder(">"), copy=False).reshape(h, -1).view(np.uint8)
    raw = np.concatenate([np.zeros((h, 1), np.uint8), rows], axis=1).tobytes()
    ihdr = struct.pack(">IIBBBBB", w, h, depth, 2, 0, 0, 0)
    return (b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", zlib.compress(raw, 6))
            + _chunk(b"IEND", b""))


def save_png(path, rgb: np.ndarray) -> None:
    Path(path).write_bytes(encode_png(rgb))


def decode_png(data: bytes) -> np.ndarray:
    """Minimal reader for truecolor 8/16-bit non-interlaced PNGs (tests and tools)."""
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError("not a PNG")
    pos, idat, hdr = 8, [], None
    while pos < len(data):
        n, tag = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif tag == b"IDAT":
            idat.append(body)
        pos += 12 + n
    w, h, depth, ctype, _, _, interlace = hdr
    if ctype != 2 or interlace != 0 or depth not in (8, 16):
        raise ValueError("decode_png supports truecolor 8/16-bit non-interlaced only")
    bpp = 3 * depth // 8
    raw = np.frombuffer(zlib.decompress(b"".join(idat)), np.uint8).reshape(h, 1 + w * bpp)
    if not raw[:, 0].any():  # every row unfiltered (what encode_png writes)
        out = raw[:, 1:].astype(np.int32)
    else:
        out = _unfilter(raw, h, w * bpp, bpp)
    img = out.astype(np.uint8)
    if depth == 16:
        return img.reshape(h, w * 3, 2).view(">u2").reshape(h, w, 3).astype(np.uint16)
    return img.reshape(h, w, 3)


def _unfilter(raw, h, stride, bpp):
    out = np.zeros((h, stride), np.int32)
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        f, line = raw[y, 0], raw[y, 1:].astype(np.int32)
        cur = np.zeros_like(line)
        for x in range(stride):
            a = cur[x - bpp] if x >= bpp else 0
            b, c = prev[x], (prev[x - bpp] if x >= bpp else 0)
            if f == 0:
                p = 0
            elif f == 1:
                p = a
            elif f == 2:
                p = b
            elif f == 3:
                p = (a + b) // 2
            else:
                pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
            cur[x] = (line[x] + p) & 0xFF
        out[y], prev = cur, cur
    return out
