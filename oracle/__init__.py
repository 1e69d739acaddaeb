"""ctypes wrapper of the CPU oracle (oracle/libbh_oracle.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package, and
only as the checker / the timed CPU baseline.  PARITY UNPINNED: see oracle/bh_oracle.c header.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

LIB_PATH = Path(__file__).resolve().parent / "libbh_oracle.so"
_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} missing: run `python -m black_hole_ray_marching_amd.build`")
        lib = C.CDLL(str(LIB_PATH))
        lib.bho_render_rows.restype = C.c_int
        lib.bho_render_rows.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                        C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                        C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_int]
        lib.bho_render_rows_variant.restype = C.c_int
        lib.bho_render_rows_variant.argtypes = lib.bho_render_rows.argtypes + [C.c_uint32]
        lib.bho_trace_ray.restype = C.c_int
        lib.bho_trace_ray.argtypes = [C.c_float * 3, C.c_float * 3, C.c_void_p, C.c_void_p, C.c_uint32,
                                      C.c_uint32, C.c_uint32, C.c_uint32, C.c_float * 3,
                                      C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_float * 6]
        lib.bho_srgb_lut.restype = None
        lib.bho_srgb_lut.argtypes = [C.c_void_p]
        lib.bho_srgb_encode.restype = C.c_uint8
        lib.bho_srgb_encode.argtypes = [C.c_float]
        lib.bho_srgb_encode_array.restype = None
        lib.bho_srgb_encode_array.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        lib.bho_bloom.restype = C.c_int
        lib.bho_bloom.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_int]
        lib.bho_srgb_table_mismatches.restype = C.c_uint64
        lib.bho_srgb_table_mismatches.argtypes = [C.c_void_p, C.c_int]
        _lib = lib
    return _lib


def render_rows(camera_uniform: bytes, uniforms: bytes, sky: np.ndarray, width: int, height: int,
                max_iters: int, scene_flags: int, row0: int = 0, row1: int | None = None,
                threads: int = 0, blackout: bool = True, row_step: int = 1, variant: int = 0):
    """Oracle render of rows row0, row0+row_step, ... < row1.  camera_uniform/uniforms: the
    112-/32-byte ABI structs.  variant: 0 = the normative arithmetic (every parity test); else
    V_* bits, the parity-envelope variants of DESIGN.md §3 (what a real WGSL driver may do instead).

    Returns (col (R,W,4) f32, blackout (R,W,4) f32 or None, n_rk (R,W) u16, fate (R,W) u8).
    """
    lib = load()
    row1 = height if row1 is None else row1
    rows = (row1 - row0 + row_step - 1) // row_step
    sky = np.ascontiguousarray(sky, dtype=np.uint8)
    col = np.empty((rows, width, 4), np.float32)
    bo = np.empty((rows, width, 4), np.float32) if blackout else None
    n_rk = np.empty((rows, width), np.uint16)
    fate = np.empty((rows, width), np.uint8)
    cam = C.create_string_buffer(bytes(camera_uniform), 112)
    uni = C.create_string_buffer(bytes(uniforms), 32)
    args = (cam, uni, sky.ctypes.data, sky.shape[1], sky.shape[0], width, height, max_iters,
            scene_flags, row0, row1, row_step, col.ctypes.data, bo.ctypes.data if bo is not None else None,
            n_rk.ctypes.data, fate.ctypes.data, threads)
    st = lib.bho_render_rows_variant(*args, variant) if variant else lib.bho_render_rows(*args)
    if st != 0:
        raise ValueError(f"bho_render_rows failed: {st}")
    return col, bo, n_rk, fate


# parity-envelope variants (oracle/bh_oracle.c BHO_V_*)
V_POW_EXP2LOG2, V_TEX_8BIT, V_TEX_NEAREST, V_ATAN2F = 1, 2, 4, 8


def trace_ray(ro0, rd0, uniforms: bytes, sky: np.ndarray, max_iters: int, scene_flags: int):
    """One explicit ray through get_col.  Returns (rgb, n_rk, fate, final ro, final rd)."""
    lib = load()
    sky = np.ascontiguousarray(sky, dtype=np.uint8)
    out = (C.c_float * 3)()
    st = (C.c_float * 6)()
    n, f = C.c_uint32(), C.c_uint32()
    uni = C.create_string_buffer(bytes(uniforms), 32)
    lib.bho_trace_ray((C.c_float * 3)(*ro0), (C.c_float * 3)(*rd0), uni, sky.ctypes.data, sky.shape[1],
                      sky.shape[0], max_iters, scene_flags, out, C.byref(n), C.byref(f), st)
    s = np.array(st, np.float32)
    return np.array(out, np.float32), int(n.value), int(f.value), s[:3], s[3:]


def srgb_encode(x: np.ndarray, threads: int = 0) -> np.ndarray:
    """Linear f32 -> sRGB byte (the Bgra8UnormSrgb store), element-wise."""
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty(x.shape, np.uint8)
    load().bho_srgb_encode_array(x.ctypes.data, out.ctypes.data, x.size, threads)
    return out


def srgb_table_mismatches(table: np.ndarray, threads: int = 0) -> int:
    t = np.ascontiguousarray(table, np.float32)
    assert t.shape == (257,)
    return int(load().bho_srgb_table_mismatches(t.ctypes.data, threads))


def bloom(col: np.ndarray, blackout: np.ndarray, levels: int = 3, threads: int = 0) -> np.ndarray:
    """bho_bloom (oracle/bh_bloom_oracle.c): the reference's Kawase bloom + remix chain on (H, W, 4)
    BGRA8 images -> the (H, W, 4) BGRA8 surface."""
    col = np.ascontiguousarray(col, np.uint8)
    blackout = np.ascontiguousarray(blackout, np.uint8)
    assert col.shape == blackout.shape and col.ndim == 3 and col.shape[2] == 4
    H, W = col.shape[:2]
    out = np.empty_like(col)
    st = load().bho_bloom(col.ctypes.data, blackout.ctypes.data, W, H, levels, out.ctypes.data, threads)
    if st != 0:
        raise ValueError(f"bho_bloom: {st}")
    return out


def srgb_lut() -> np.ndarray:
    out = np.empty(256, np.float32)
    load().bho_srgb_lut(out.ctypes.data)
    return out
