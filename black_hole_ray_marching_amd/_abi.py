"""ctypes view of include/bh_render.h (the C ABI).  No torch types cross this boundary."""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(os.environ.get("BH_LIB", Path(__file__).resolve().parent / "libbh_render.so"))

BH_OK = 0
BH_ERR_INVALID_ARG = -1
BH_ERR_UNSUPPORTED = -2
BH_ERR_HIP = -3
BH_ERR_NO_DEVICE = -4
BH_ERR_OUT_OF_MEMORY = -5
BH_ERR_INTERNAL = -6

BH_OUT_RGBA32F, BH_OUT_RGBA16F, BH_OUT_BGRA8_SRGB = 0, 1, 2
BH_BLOOM_AUTO, BH_BLOOM_LITERAL = 0, 1
BH_MATH_EXACT, BH_MATH_FAST = 0, 1
BH_SCENE_DISC, BH_SCENE_MARKERS = 1, 2
BH_SCENE_DEFAULT = 3
BH_LAYOUT_ROWMAJOR, BH_LAYOUT_TILES, BH_LAYOUT_TILES_RGB, BH_LAYOUT_TILES_RGBM, BH_LAYOUT_TILES_RGBM14 = 0, 1, 2, 3, 4
BH_UNPACK_RGBM14 = 0x100  # format flag of the RGBM unpacks: the shards are BH_LAYOUT_TILES_RGBM14
BH_ORDER_STATES = 32
BH_BLOOM_SETS = 4
BH_MAX_FRAMES = 256
BH_SCHED_TILE, BH_SCHED_PAIR, BH_SCHED_PERSISTENT = 0, 1, 2
BH_SCHED_FLAG_STATIC_ORDER = 0x100
BH_SCHED_FLAG_ISSUE_ORDER = 0x200   # exact math: force the source-order build of the kernels
BH_SCHED_FLAG_LATENCY = 0x400       # exact math: force the machine-scheduled build
BH_FATE_CAP, BH_FATE_ESCAPE, BH_FATE_SURFACE, BH_FATE_BLACKOUT = 0, 1, 2, 3
BH_TILE = 8

ABI_VERSION = 8

BYTES_PER_PIXEL = {BH_OUT_RGBA32F: 16, BH_OUT_RGBA16F: 8, BH_OUT_BGRA8_SRGB: 4}


class bh_camera_uniform(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("_pad0", C.c_float),
                ("screen_tri", (C.c_float * 4) * 3), ("world_tri", (C.c_float * 4) * 3)]


class bh_uniforms(C.Structure):
    _fields_ = [("rs", C.c_float), ("delta_time_mult", C.c_float), ("bg_brightness", C.c_float),
                ("blackout_eh", C.c_uint32), ("max_dist", C.c_float), ("distortion_power", C.c_float),
                ("_pad", C.c_uint32 * 2)]


class bh_camera(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("dir", C.c_float * 3), ("up", C.c_float * 3),
                ("aspect", C.c_float), ("fovy", C.c_float), ("znear", C.c_float), ("zfar", C.c_float)]


class bh_controller(C.Structure):
    _fields_ = [(n, C.c_uint8) for n in ("forward", "backward", "left", "right", "up", "down", "pan_up",
                                          "pan_down", "pan_left", "pan_right", "exp_towards_origin",
                                          "exp_away_origin", "mouse_pressed", "has_prev_cursor",
                                          "has_curr_cursor", "_pad")] + \
              [("prev_cursor", C.c_float * 2), ("curr_cursor", C.c_float * 2), ("speed", C.c_float),
               ("pan_speed", C.c_float)]


class bh_render_desc(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("max_iters", C.c_uint32),
                ("scene_flags", C.c_uint32), ("format", C.c_uint32), ("math", C.c_uint32),
                ("layout", C.c_uint32), ("shard_index", C.c_uint32), ("shard_count", C.c_uint32),
                ("schedule", C.c_uint32), ("out_col", C.c_void_p), ("out_blackout", C.c_void_p),
                ("dbg_n_rk", C.c_void_p), ("dbg_fate", C.c_void_p),
                ("dbg_steps", C.c_void_p), ("partition", C.c_void_p)]


class bh_presenter_desc(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("width", "height", "max_iters", "scene_flags", "math", "levels", "batch",
                                          "bloom_cus", "depth", "march_streams")]


BH_PRESENT_BATCH_MAX = 32
BH_PRESENT_DEPTH_MAX = 8

assert C.sizeof(bh_camera_uniform) == 112
assert C.sizeof(bh_uniforms) == 32

# name -> (restype, argtypes): every entry point declared in include/bh_render.h
SIGNATURES = {
    "bh_abi_version": (C.c_int, []),
    "bh_status_string": (C.c_char_p, [C.c_int]),
    "bh_last_error": (C.c_char_p, []),
    "bh_uniforms_default": (C.c_int, [C.POINTER(bh_uniforms)]),
    "bh_camera_default": (C.c_int, [C.c_uint32, C.c_uint32, C.POINTER(bh_camera)]),
    "bh_camera_uniform_update": (C.c_int, [C.POINTER(bh_camera), C.POINTER(bh_camera_uniform)]),
    "bh_camera_look_at": (C.c_int, [C.c_float * 3, C.c_float * 3, C.c_uint32, C.c_uint32, C.POINTER(bh_camera)]),
    "bh_synthetic_sky": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64]),
    "bh_create": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.POINTER(C.c_void_p)]),
    "bh_destroy": (C.c_int, [C.c_void_p]),
    "bh_render": (C.c_int, [C.c_void_p, C.POINTER(bh_camera_uniform), C.POINTER(bh_uniforms),
                            C.POINTER(bh_render_desc), C.c_void_p]),
    "bh_render_frames": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(bh_camera_uniform), C.POINTER(bh_uniforms),
                                   C.POINTER(bh_render_desc), C.c_void_p]),
    "bh_shard_tile_count": (C.c_int64, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "bh_tiles_unpack": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                  C.c_uint64, C.c_uint32, C.c_void_p]),
    "bh_tiles_unpack_rgb": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.c_uint64, C.c_uint32, C.c_void_p]),
    "bh_tiles_unpack_rgb_rows": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                           C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p]),
    "bh_tiles_unpack_rgbm": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                       C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p]),
    "bh_tile_bytes": (C.c_int64, [C.c_uint32, C.c_uint32]),
    "bh_partition_create": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.c_int,
                                      C.POINTER(C.c_void_p)]),
    "bh_partition_destroy": (C.c_int, [C.c_void_p]),
    "bh_partition_tile_count": (C.c_int64, [C.c_void_p, C.c_uint32]),
    "bh_partition_map": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.c_void_p,
                                   C.c_void_p]),
    "bh_tiles_unpack_rgbm_partition": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                                 C.c_uint32, C.c_uint32, C.c_void_p]),
    "bh_srgb_encode_table": (C.c_int, [C.c_void_p]),
    "bh_controller_update": (C.c_int, [C.POINTER(bh_controller), C.POINTER(bh_camera), C.c_float, C.c_int,
                                       C.POINTER(C.c_int)]),
    "bh_bloom": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                           C.c_void_p, C.c_void_p]),
    "bh_bloom_check": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64), C.c_char_p,
                                 C.c_size_t]),
    "bh_presenter_create": (C.c_int, [C.c_void_p, C.POINTER(bh_presenter_desc), C.POINTER(C.c_void_p)]),
    "bh_presenter_destroy": (C.c_int, [C.c_void_p]),
    "bh_present_frames": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(bh_camera_uniform), C.POINTER(bh_uniforms),
                                    C.POINTER(C.c_void_p), C.c_void_p]),
    "bh_present": (C.c_int, [C.c_void_p, C.POINTER(bh_camera_uniform), C.POINTER(bh_uniforms), C.c_void_p, C.c_void_p]),
    "bh_bloom_plan_failures": (C.c_int64, [C.c_char_p, C.c_size_t]),
    "bh_selftest_crmath": (C.c_int, [C.c_int, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64), C.c_void_p, C.c_int]),
    "bh_set_clock_probe": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "bh_graph_release": (C.c_int, [C.c_void_p]),
}

_lib = None


def load() -> C.CDLL:
    """Load libbh_render.so.  Fails loudly if it has not been built (there is no fallback path).

    torch is imported first when available so that this library binds to the same HIP runtime
    (SONAME libamdhip64.so.7) that torch already mapped; otherwise two runtimes would coexist.
    """
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(f"{LIB_PATH} is missing: run `python -m black_hole_ray_marching_amd.build` "
                           "(there is no CPU fallback for the render path)")
    if os.environ.get("BH_NO_TORCH_PRELOAD") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    lib = C.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        if "BH_LIB" in os.environ and not hasattr(lib, name):
            continue  # development override (A/B of an older build): bind what it exports
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.bh_abi_version() != ABI_VERSION:
        raise RuntimeError("libbh_render.so ABI version mismatch")
    _lib = lib
    return lib


class BhError(RuntimeError):
    def __init__(self, status: int, what: str):
        lib = load()
        msg = lib.bh_status_string(status).decode()
        detail = lib.bh_last_error().decode()
        super().__init__(f"{what}: {msg} ({status})" + (f": {detail}" if detail else ""))
        self.status = status


def check(status: int, what: str) -> None:
    if status != BH_OK:
        raise BhError(status, what)
