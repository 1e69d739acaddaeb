"""MI355X-native geodesic ray-marcher: drop-in for the `Scene::render` hot path of
jonathandw743/black_hole_ray_marching (src/black_hole_maybe.wgsl get_col / fs_main).

The compute path is libbh_render.so (hand-written HIP for gfx950 behind the C ABI of
include/bh_render.h); this package is the host-side mirror of the reference's Scene/Camera API.
"""
from ._abi import (BH_BLOOM_AUTO, BH_BLOOM_LITERAL, BH_FATE_BLACKOUT, BH_FATE_CAP, BH_FATE_ESCAPE, BH_FATE_SURFACE, BH_LAYOUT_ROWMAJOR,
                   BH_LAYOUT_TILES, BH_LAYOUT_TILES_RGB, BH_LAYOUT_TILES_RGBM, BH_LAYOUT_TILES_RGBM14, BH_UNPACK_RGBM14, BH_ORDER_STATES, BH_BLOOM_SETS, BH_MAX_FRAMES, BH_MATH_EXACT, BH_MATH_FAST, BH_OUT_BGRA8_SRGB, BH_OUT_RGBA16F,
                   BH_OUT_RGBA32F, BH_SCENE_DEFAULT, BH_SCENE_DISC, BH_SCENE_MARKERS, BH_SCHED_FLAG_STATIC_ORDER, BH_SCHED_FLAG_ISSUE_ORDER, BH_SCHED_FLAG_LATENCY, BH_SCHED_PAIR, BH_SCHED_PERSISTENT, BH_SCHED_TILE,
                   BYTES_PER_PIXEL,
                   BhError, load)
from .scene import (MAX_ITERATIONS, Camera, CameraController, CameraUniform, FrameBatch, Partition, Presenter, Scene, Uniforms, bloom_check, bloom_plan_failures, clock_mhz, load_sky,
                    partition_map, shard_tile_count, srgb_encode_table, tiles_unpack_rgbm_partition,
                    synthetic_sky, tile_bytes, tiles_unpack, tiles_unpack_rgb, tiles_unpack_rgbm)

__version__ = "0.4.0"
