"""Minimal PNG writer for offline frames ("a PNG writer for offline frames"):
8-bit RGBA, no filtering, zlib-compressed IDAT.  Takes the BGRA8 surface bh_bloom / bh_render write."""
from __future__ import annotations

import struct
import zlib
from pathlib import Path

import numpy as np


def _chunk(tag: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def encode_png(bgra: np.ndarray, level: int = 6) -> bytes:
    """(H, W, 4) uint8 BGRA (the Bgra8UnormSrgb byte order) -> PNG bytes (sRGB RGBA8)."""
    a = np.ascontiguousarray(bgra, np.uint8)
    if a.ndim != 3 or a.shape[2] != 4:
        raise ValueError("expected (H, W, 4) uint8")
    h, w = a.shape[:2]
    rgba = a[..., [2, 1, 0, 3]]
    raw = np.concatenate([np.zeros((h, 1), np.uint8), rgba.reshape(h, w * 4)], axis=1)  # filter 0 per row
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)
    srgb = bytes([0])  # sRGB chunk: perceptual intent
    return (b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + _chunk(b"sRGB", srgb) +
            _chunk(b"IDAT", zlib.compress(raw.tobytes(), level)) + _chunk(b"IEND", b""))


def decode_png_rgba(data: bytes) -> np.ndarray:
    """Inverse of encode_png for its own output (filter 0, RGBA8): used by the tests."""
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        tag, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            w, h = struct.unpack(">II", body[:8])
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + w * 4)
    assert (raw[:, 0] == 0).all()
    return raw[:, 1:].reshape(h, w, 4)


def write_png(path, bgra: np.ndarray) -> None:
    Path(path).write_bytes(encode_png(bgra))
