"""Host-side mirror of the reference's render-to-texture interface, over the C ABI.

Reference (jonathandw743/black_hole_ray_marching):
  Camera            src/camera.rs:11-20, 56-112
  CameraUniform     src/uniforms.rs:98-133
  OtherUniforms     src/otheruniforms.rs:105-118, defaults src/scene.rs:89-137
  Scene             src/scene.rs:28-522  (new :53, resize :370, update :444, render :470)

`Scene.render(output, blackout_output=None)` mirrors `Scene::render(encoder, output_view,
blackout_output_view)`: the caller owns the output images (device tensors here, texture views
there); `None` for the blackout target mirrors `Option::None`.  Errors raise `BhError` (the
reference panics on wgpu validation errors).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _abi
from ._abi import (BH_LAYOUT_ROWMAJOR, BH_LAYOUT_TILES, BH_LAYOUT_TILES_RGB, BH_LAYOUT_TILES_RGBM, BH_LAYOUT_TILES_RGBM14, BH_UNPACK_RGBM14, BH_MATH_EXACT, BH_MATH_FAST, BH_OUT_RGBA16F,
                   BH_OUT_RGBA32F, BH_OUT_BGRA8_SRGB, BH_SCENE_DEFAULT, BYTES_PER_PIXEL, BhError, check, load)

MAX_ITERATIONS = 1000  # src/black_hole_maybe.wgsl:85


@dataclass
class Camera:
    """src/camera.rs:11-20."""
    pos: tuple = (0.0, 0.0, -20.0)
    dir: tuple = (0.0, 0.0, 1.0)
    up: tuple = (0.0, 1.0, 0.0)
    aspect: float = 1.0
    fovy: float = float(np.float32(np.pi) * np.float32(0.5))
    znear: float = 0.1
    zfar: float = 100.0

    @classmethod
    def default(cls, width: int, height: int) -> "Camera":
        """The camera of Scene::new (src/scene.rs:68-76)."""
        c = _abi.bh_camera()
        check(load().bh_camera_default(width, height, C.byref(c)), "bh_camera_default")
        return cls._from_c(c)

    @classmethod
    def look_at(cls, pos, target, width: int, height: int) -> "Camera":
        c = _abi.bh_camera()
        check(load().bh_camera_look_at((C.c_float * 3)(*pos), (C.c_float * 3)(*target), width, height,
                                       C.byref(c)), "bh_camera_look_at")
        return cls._from_c(c)

    @classmethod
    def _from_c(cls, c) -> "Camera":
        return cls(tuple(c.pos), tuple(c.dir), tuple(c.up), c.aspect, c.fovy, c.znear, c.zfar)

    def to_c(self) -> _abi.bh_camera:
        return _abi.bh_camera((C.c_float * 3)(*self.pos), (C.c_float * 3)(*self.dir),
                              (C.c_float * 3)(*self.up), self.aspect, self.fovy, self.znear, self.zfar)


class CameraController:
    """CameraController (src/camera.rs:115-366): key state, speeds and cursor -> camera motion.
    `process_key` takes the reference's key names (process_event :186-261); `update_camera` is
    update_camera (:280-366) through the C ABI (glam f32 arithmetic).  Driving it with a scripted key
    sequence gives the camera paths of an offline, multi-frame render (tools/render_path.py)."""

    KEYS = {"W": "forward", "S": "backward", "A": "left", "D": "right", "Space": "up", "F": "down",
            "ArrowUp": "pan_up", "ArrowDown": "pan_down", "ArrowLeft": "pan_left", "ArrowRight": "pan_right",
            "P": "exp_towards_origin", "O": "exp_away_origin"}

    def __init__(self, speed: float = 5.0, pan_speed: float = 0.5) -> None:  # src/scene.rs:78
        self.c = _abi.bh_controller()
        self.c.speed, self.c.pan_speed = speed, pan_speed

    def process_key(self, key: str, pressed: bool) -> bool:
        if key == "Q":
            if pressed:
                self.c.speed = float(np.float32(self.c.speed) / np.float32(1.5))
            return True
        if key == "E":
            if pressed:
                self.c.speed = float(np.float32(self.c.speed) * np.float32(1.5))
            return True
        if key not in self.KEYS:
            return False
        setattr(self.c, self.KEYS[key], 1 if pressed else 0)
        return True

    def process_mouse(self, pressed: bool) -> None:
        self.c.mouse_pressed = 1 if pressed else 0

    def process_cursor(self, x: float, y: float) -> None:
        """CursorMoved: prev <- curr, curr <- (x, y) (as f32)."""
        self.c.prev_cursor[0], self.c.prev_cursor[1] = self.c.curr_cursor[0], self.c.curr_cursor[1]
        self.c.has_prev_cursor = self.c.has_curr_cursor
        self.c.curr_cursor[0], self.c.curr_cursor[1] = float(np.float32(x)), float(np.float32(y))
        self.c.has_curr_cursor = 1

    def update_camera(self, camera: "Camera", dt: float, do_pan: bool = False) -> tuple["Camera", bool]:
        cc = camera.to_c()
        moved = C.c_int(0)
        check(load().bh_controller_update(C.byref(self.c), C.byref(cc), float(np.float32(dt)), int(do_pan),
                                          C.byref(moved)), "bh_controller_update")
        return Camera._from_c(cc), bool(moved.value)


class CameraUniform:
    """src/uniforms.rs:98-133 — the 112-byte WGSL `Camera` uniform."""

    def __init__(self) -> None:
        self.c = _abi.bh_camera_uniform()
        for i, (x, y) in enumerate(((3.0, 1.0), (-1.0, 1.0), (-1.0, -3.0))):  # ::new
            self.c.screen_tri[i][0], self.c.screen_tri[i][1] = x, y

    def update(self, camera: Camera) -> None:
        check(load().bh_camera_uniform_update(C.byref(camera.to_c()), C.byref(self.c)),
              "bh_camera_uniform_update")

    @property
    def pos(self) -> np.ndarray:
        return np.array(self.c.pos, dtype=np.float32)

    @property
    def world_tri(self) -> np.ndarray:
        return np.array([[self.c.world_tri[i][k] for k in range(3)] for i in range(3)], dtype=np.float32)

    def to_bytes(self) -> bytes:
        return bytes(self.c)


@dataclass
class Uniforms:
    """The 32-byte WGSL `Uniforms` block (src/black_hole_maybe.wgsl:58-69) with Scene::new defaults."""
    rs: float = 1.0
    delta_time_mult: float = 0.5
    bg_brightness: float = 0.5
    blackout_eh: int = 1   # PodBool::r#false() stores inner = 1 (src/podbool.rs:24-26) => on
    max_dist: float = 250.0
    distortion_power: float = 1.0

    @classmethod
    def default(cls) -> "Uniforms":
        u = _abi.bh_uniforms()
        check(load().bh_uniforms_default(C.byref(u)), "bh_uniforms_default")
        return cls(u.rs, u.delta_time_mult, u.bg_brightness, u.blackout_eh, u.max_dist, u.distortion_power)

    def to_c(self) -> _abi.bh_uniforms:
        return _abi.bh_uniforms(self.rs, self.delta_time_mult, self.bg_brightness, int(self.blackout_eh),
                                self.max_dist, self.distortion_power)

    def as_dict(self) -> dict:
        return dict(rs=self.rs, delta_time_mult=self.delta_time_mult, blackout_eh=self.blackout_eh,
                    max_dist=self.max_dist, distortion_power=self.distortion_power)


def synthetic_sky(width: int = 4096, height: int = 2048, seed: int = 0x5EED_B1AC_401E) -> np.ndarray:
    """Deterministic RGBA8 sRGB equirectangular sky, (height, width, 4) uint8."""
    out = np.empty((height, width, 4), dtype=np.uint8)
    check(load().bh_synthetic_sky(out.ctypes.data, width, height, seed), "bh_synthetic_sky")
    return out


def load_sky(path) -> np.ndarray:
    """Texture::from_bytes / from_image (src/texture.rs:11-27, src/scene.rs:186-194): decode an image
    file (the reference ships src/space_4096x2048.jpg) to (H, W, 4) RGBA8 with alpha 255, the bytes
    bh_create uploads as the Rgba8UnormSrgb sky.  Decoded with Pillow (libjpeg-turbo); the reference
    uses the jpeg-decoder crate 0.3.1, and JPEG decoders legitimately differ by +-1 LSB, so the
    texels -- an input to both renderers -- are not part of kernel parity."""
    from PIL import Image
    with Image.open(path) as im:
        return np.ascontiguousarray(np.asarray(im.convert("RGBA"), dtype=np.uint8))


def srgb_encode_table() -> np.ndarray:
    """The 257 thresholds of the BGRA8 sRGB encoder (bh_srgb.hpp): code(x) = max k with x >= T[k]."""
    out = np.empty(257, np.float32)
    check(load().bh_srgb_encode_table(out.ctypes.data), "bh_srgb_encode_table")
    return out


def shard_tile_count(width: int, height: int, shard_index: int, shard_count: int) -> int:
    n = load().bh_shard_tile_count(width, height, shard_index, shard_count)
    if n < 0:
        raise BhError(int(n), "bh_shard_tile_count")
    return int(n)


def bloom_check(width: int, height: int, levels: int = 3, schedule: int = 0) -> list[tuple]:
    """bh_bloom_check (host only, no device): plan bh_bloom's chain for this frame size and check every
    launch's index arithmetic on the host (DESIGN.md §7b "Bound checks"); raises BhError on a violation.
    Returns the chain's launches as (form, ow, oh, tw, th, rx, ry) tuples, in launch order."""
    lib = load()
    n = C.c_uint64()
    buf = C.create_string_buffer(1 << 16)
    check(lib.bh_bloom_check(width, height, levels, schedule, C.byref(n), buf, len(buf)), "bh_bloom_check")
    out = []
    for line in buf.value.decode().splitlines():
        f = line.split()
        out.append((f[0], *map(int, f[1:])))
    return out


def bloom_plan_failures() -> tuple[int, str]:
    """bh_bloom_plan_failures: (plans real bh_bloom calls built whose host check refused them -- each such pass
    ran its general kernel, same bytes, slower -- process-wide, the last refusal's message)."""
    buf = C.create_string_buffer(512)
    n = load().bh_bloom_plan_failures(buf, len(buf))
    return int(n), buf.value.decode()


def _ptr(t) -> int | None:
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def tile_bytes(layout: int, fmt: int) -> int:
    """Bytes of one 8x8 tile of a BH_LAYOUT_TILES* layout in format `fmt` (bh_tile_bytes)."""
    n = load().bh_tile_bytes(layout, fmt)
    if n < 0:
        raise BhError(int(n), "bh_tile_bytes")
    return int(n)


def _check_size(t, need: int, name: str, what: str = "render") -> None:
    """Host-side bounds check of a caller buffer (tensor-like objects; raw pointers are trusted)."""
    if t is None or isinstance(t, int) or not hasattr(t, "element_size"):
        return
    have = t.numel() * t.element_size()
    if have < need:
        raise BhError(_abi.BH_ERR_INVALID_ARG, f"{what}: {name} holds {have} bytes, needs {need}")
    if hasattr(t, "is_contiguous") and not t.is_contiguous():
        raise BhError(_abi.BH_ERR_INVALID_ARG, f"{what}: {name} must be contiguous")


class FrameBatch:
    """A prepared bh_render_frames call (Scene.prepare_frames): its targets stay referenced, so the
    device pointers in its descriptors stay valid while the batch lives."""

    def __init__(self, scene: "Scene", descs, keep) -> None:
        self.scene, self.descs, self._keep = scene, descs, keep
        self.n = len(descs)
        self._cams = (_abi.bh_camera_uniform * self.n)()

    def render(self, n: int | None = None, cameras=None, stream=None) -> None:
        """Render the first `n` frames (default all) with cameras[i] (default: the scene's camera) and
        the scene's current uniforms."""
        n = self.n if n is None else n
        if not 1 <= n <= self.n:
            raise BhError(_abi.BH_ERR_INVALID_ARG, f"FrameBatch.render: 1..{self.n} frames, got {n}")
        sc = self.scene
        if cameras is None:
            cameras = [sc.camera_uniform] * n
        elif len(cameras) != n:
            raise BhError(_abi.BH_ERR_INVALID_ARG, "render_frames: per-frame lists must have one entry per frame")
        for i, c in enumerate(cameras):
            self._cams[i] = c.c
        check(sc.lib.bh_render_frames(sc._ctx, n, self._cams, C.byref(sc.uniforms.to_c()), self.descs,
                                      _stream_handle(stream)), "bh_render_frames")


class Scene:
    """src/scene.rs `Scene`: owns the sky texture (on `device`), camera, uniforms; renders frames."""

    def __init__(self, width: int, height: int, sky: np.ndarray | None = None, device: int = 0,
                 render_blackout: bool = True, max_iters: int = MAX_ITERATIONS,
                 scene_flags: int = BH_SCENE_DEFAULT, math: int = BH_MATH_FAST) -> None:
        self.lib = load()
        self.width, self.height = width, height
        self.render_blackout = render_blackout
        self.max_iters, self.scene_flags, self.math = max_iters, scene_flags, math
        self.camera = Camera.default(width, height)
        self.camera_uniform = CameraUniform()
        self.camera_uniform.update(self.camera)
        self.uniforms = Uniforms.default()
        if sky is None:
            sky = synthetic_sky()
        sky = np.ascontiguousarray(sky, dtype=np.uint8)
        if sky.ndim != 3 or sky.shape[2] != 4:
            raise ValueError("sky must be (H, W, 4) uint8 RGBA (Rgba8UnormSrgb texels)")
        self.sky = sky
        ctx = C.c_void_p()
        check(self.lib.bh_create(sky.ctypes.data, sky.shape[1], sky.shape[0], device, C.byref(ctx)), "bh_create")
        self._ctx = ctx
        self.device = device

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self.lib.bh_destroy(self._ctx)
            self._ctx = None
        self._clock_acc = None

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:
            pass

    def resize(self, width: int, height: int) -> None:
        """src/scene.rs:370-382: only the aspect changes; corners are re-derived by update()."""
        self.width, self.height = width, height
        self.camera.aspect = float(np.float32(width) / np.float32(height))

    def update(self, camera: Camera | None = None) -> None:
        """src/scene.rs:444-466 (minus the interactive controller): re-derive the camera uniform."""
        if camera is not None:
            self.camera = camera
        self.camera_uniform.update(self.camera)

    def _desc(self, output, blackout_output, fmt, dbg_n_rk, dbg_fate, math, layout, shard_index, shard_count,
              width, height, schedule, dbg_steps, partition=None) -> _abi.bh_render_desc:
        if output is None:
            raise BhError(_abi.BH_ERR_INVALID_ARG, "render: output is required")
        if not self.render_blackout and blackout_output is not None:
            raise BhError(_abi.BH_ERR_INVALID_ARG, "render: scene built without a blackout target")
        d = _abi.bh_render_desc()
        d.width, d.height = width or self.width, height or self.height
        d.max_iters, d.scene_flags = self.max_iters, self.scene_flags
        d.format = fmt
        d.math = self.math if math is None else math
        d.layout, d.shard_index, d.shard_count = layout, shard_index, shard_count
        d.schedule = schedule
        bpp = _abi.BYTES_PER_PIXEL.get(fmt, 0)
        if layout == BH_LAYOUT_ROWMAJOR:
            px = d.width * d.height
            col_bytes = px * bpp
        else:
            if partition is not None:
                if (partition.width, partition.height, partition.shard_count) != (d.width, d.height, shard_count):
                    raise BhError(_abi.BH_ERR_INVALID_ARG, "render: the partition's frame size / shard count differ")
                d.partition = partition.handle
                nt = partition.tile_count(shard_index)
            else:
                nt = shard_tile_count(d.width, d.height, shard_index, shard_count)
            px = nt * 64
            col_bytes = nt * tile_bytes(layout, fmt) if bpp and layout <= BH_LAYOUT_TILES_RGBM14 else px * bpp
        _check_size(output, col_bytes, "output")
        _check_size(blackout_output, col_bytes, "blackout_output")
        _check_size(dbg_n_rk, px * 2, "dbg_n_rk")
        _check_size(dbg_fate, px, "dbg_fate")
        _check_size(dbg_steps, px * 2, "dbg_steps")
        d.out_col, d.out_blackout = _ptr(output), _ptr(blackout_output)
        d.dbg_n_rk, d.dbg_fate, d.dbg_steps = _ptr(dbg_n_rk), _ptr(dbg_fate), _ptr(dbg_steps)
        return d

    def render(self, output, blackout_output=None, *, fmt: int = BH_OUT_RGBA32F, stream=None,
               dbg_n_rk=None, dbg_fate=None, math: int | None = None, layout: int = BH_LAYOUT_ROWMAJOR,
               shard_index: int = 0, shard_count: int = 1, width: int | None = None,
               height: int | None = None, schedule: int = 0, dbg_steps=None, partition=None) -> None:
        """Scene::render (src/scene.rs:470-522): one pass writing `col` and optionally `blackout_col`.

        `output`/`blackout_output`: caller-owned device buffers (torch tensors or raw pointers).
        Asynchronous on `stream` (a torch.cuda.Stream, a raw hipStream_t int, or None = current).
        """
        d = self._desc(output, blackout_output, fmt, dbg_n_rk, dbg_fate, math, layout, shard_index, shard_count,
                       width, height, schedule, dbg_steps, partition)
        check(self.lib.bh_render(self._ctx, C.byref(self.camera_uniform.c), C.byref(self.uniforms.to_c()),
                                 C.byref(d), _stream_handle(stream)), "bh_render")

    def render_frames(self, outputs, blackout_outputs=None, *, cameras=None, fmt: int = BH_OUT_RGBA32F, stream=None,
                      dbg_n_rk=None, dbg_fate=None, dbg_steps=None, math: int | None = None,
                      layout: int = BH_LAYOUT_ROWMAJOR, shard_index: int = 0, shard_count: int = 1,
                      width: int | None = None, height: int | None = None, schedule: int = 0,
                      partition=None) -> None:
        """Several frames in one launch (bh_render_frames, up to BH_MAX_FRAMES): frame i renders with
        cameras[i] (CameraUniform; default: this scene's camera for every frame) into outputs[i] /
        blackout_outputs[i]; each frame's result is exactly render()'s."""
        self.prepare_frames(outputs, blackout_outputs, fmt=fmt, dbg_n_rk=dbg_n_rk, dbg_fate=dbg_fate,
                            dbg_steps=dbg_steps, math=math, layout=layout, shard_index=shard_index,
                            shard_count=shard_count, width=width, height=height, schedule=schedule,
                            partition=partition).render(cameras=cameras, stream=stream)

    def prepare_frames(self, outputs, blackout_outputs=None, *, fmt: int = BH_OUT_RGBA32F, dbg_n_rk=None,
                       dbg_fate=None, dbg_steps=None, math: int | None = None, layout: int = BH_LAYOUT_ROWMAJOR,
                       shard_index: int = 0, shard_count: int = 1, width: int | None = None,
                       height: int | None = None, schedule: int = 0, partition=None) -> "FrameBatch":
        """A render_frames call prepared once for targets that are rendered into again and again (an
        offline camera path, the bench): the descriptors are validated and built here, and each
        FrameBatch.render is one bh_render_frames call -- at 256x256 a launch of 32 frames takes ~0.2
        ms on the GPU, less than building 32 descriptors in Python."""
        n = len(outputs)
        if not 1 <= n <= _abi.BH_MAX_FRAMES:
            raise BhError(_abi.BH_ERR_INVALID_ARG, f"render_frames: 1..{_abi.BH_MAX_FRAMES} frames, got {n}")
        per = lambda v: v if v is not None else [None] * n  # noqa: E731
        bos, nrks, fates, steps = per(blackout_outputs), per(dbg_n_rk), per(dbg_fate), per(dbg_steps)
        if not (len(bos) == len(nrks) == len(fates) == len(steps) == n):
            raise BhError(_abi.BH_ERR_INVALID_ARG, "render_frames: per-frame lists must have one entry per frame")
        descs = (_abi.bh_render_desc * n)(*[self._desc(outputs[i], bos[i], fmt, nrks[i], fates[i], math, layout,
                                                       shard_index, shard_count, width, height, schedule, steps[i],
                                                       partition)
                                            for i in range(n)])
        return FrameBatch(self, descs, (outputs, blackout_outputs, dbg_n_rk, dbg_fate, dbg_steps, partition))

    def set_clock_probe(self, acc, stride: int = 256) -> None:
        """bh_set_clock_probe: arm (acc = a zeroed device buffer of 128 u64) or disarm (acc = None) the
        shader-clock sampling of this scene's march launches; clock_mhz() reads the result."""
        if acc is not None:
            _check_size(acc, 128 * 8, "acc", "set_clock_probe")
        check(self.lib.bh_set_clock_probe(self._ctx, _ptr(acc), stride), "bh_set_clock_probe")
        # the armed ctx holds acc's raw pointer: keep the tensor alive until disarmed (or close), so the
        # caching allocator cannot hand its memory to another tensor while march launches add into it
        self._clock_acc = acc

    def graph_release(self) -> None:
        """bh_graph_release: unpin the order states and bloom scratch sets that stream captures marked
        (call it after destroying every graph captured from this scene)."""
        check(self.lib.bh_graph_release(self._ctx), "bh_graph_release")

    def bloom(self, col, blackout, out, *, levels: int = 3, schedule: int = 0, width: int | None = None,
              height: int | None = None, stream=None) -> None:
        """Bloom::render (src/bloom.rs:53-71): the Kawase bloom + remix chain over this scene's two
        BGRA8-sRGB targets (render with fmt=BH_OUT_BGRA8_SRGB) into `out` (the surface).  levels=3 is
        the reference's (src/state.rs:125)."""
        if col is None or blackout is None or out is None:
            raise BhError(_abi.BH_ERR_INVALID_ARG, "bloom: col, blackout and out are required")
        need = (width or self.width) * (height or self.height) * 4
        for t, name in ((col, "col"), (blackout, "blackout"), (out, "out")):
            _check_size(t, need, name, "bloom")
        check(self.lib.bh_bloom(self._ctx, _ptr(col), _ptr(blackout), width or self.width, height or self.height,
                                levels, schedule, _ptr(out), _stream_handle(stream)), "bh_bloom")


class Presenter:
    """bh_presenter (include/bh_render.h): the frame the reference app presents per redraw -- State::render
    (src/state.rs:270-286): Scene::render into the two Bgra8UnormSrgb targets, then Bloom::render to the
    surface -- pipelined: a call's frames march while the previous call's are bloomed on a second stream, and
    (march_streams 2) while the previous call's march tail still runs on the other march stream.
    Every surface equals scene.render(..., fmt=BH_OUT_BGRA8_SRGB) + scene.bloom(...) bytes."""

    def __init__(self, scene: "Scene", width: int | None = None, height: int | None = None, *, levels: int = 3,
                 batch: int = 1, bloom_cus: int = 0, depth: int = 0, march_streams: int = 0,
                 max_iters: int | None = None, math: int | None = None) -> None:
        self.scene = scene
        self.width, self.height = width or scene.width, height or scene.height
        self.batch = batch
        d = _abi.bh_presenter_desc(self.width, self.height, max_iters or scene.max_iters, scene.scene_flags,
                                   scene.math if math is None else math, levels, batch, bloom_cus, depth, march_streams)
        h = C.c_void_p()
        check(scene.lib.bh_presenter_create(scene._ctx, C.byref(d), C.byref(h)), "bh_presenter_create")
        self.handle = h
        self._cams = (_abi.bh_camera_uniform * batch)()
        self._outs = (C.c_void_p * batch)()
        self._keep = None

    def present(self, surfaces, cameras=None, stream=None) -> None:
        """Frames cameras[i] (CameraUniform; default: the scene's camera) -> surfaces[i] (width x height BGRA8
        device images), len(surfaces) <= batch; asynchronous on `stream` (the stream then waits for them)."""
        n = len(surfaces)
        if not 1 <= n <= self.batch:
            raise BhError(_abi.BH_ERR_INVALID_ARG, f"present: 1..{self.batch} surfaces, got {n}")
        if cameras is None:
            cameras = [self.scene.camera_uniform] * n
        elif len(cameras) != n:
            raise BhError(_abi.BH_ERR_INVALID_ARG, "present: one camera per surface")
        for i, (c, t) in enumerate(zip(cameras, surfaces)):
            _check_size(t, self.width * self.height * 4, "surface", "present")
            self._cams[i] = c.c
            self._outs[i] = _ptr(t)
        self._keep = surfaces  # referenced until the next call (the stream orders their later users)
        check(self.scene.lib.bh_present_frames(self.handle, n, self._cams, C.byref(self.scene.uniforms.to_c()),
                                               self._outs, _stream_handle(stream)), "bh_present_frames")

    def close(self) -> None:
        if getattr(self, "handle", None):
            self.scene.lib.bh_presenter_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def clock_mhz(acc) -> dict:
    """The shader clock sampled by set_clock_probe: acc (128 u64 as an int64 array) -> per-XCD MHz and
    the clock over all sampled waves (100 MHz * shader ticks / reference ticks)."""
    a = np.asarray(acc, dtype=np.int64).view(np.uint64).reshape(8, 16)
    ticks, ref, waves = a[:, 0].astype(np.float64), a[:, 1].astype(np.float64), a[:, 2].astype(np.int64)
    per = [round(100.0 * t / r, 1) if r > 0 else None for t, r in zip(ticks, ref)]
    tot = float(ref.sum())
    return {"mhz": round(100.0 * float(ticks.sum()) / tot, 1) if tot > 0 else None,
            "per_xcd_mhz": per, "waves": int(waves.sum()),
            "wave_ms": round(tot / 1e5 / max(1, int(waves.sum())), 5)}


def _stream_handle(stream) -> int | None:
    if stream is None:
        try:
            import torch
            if torch.cuda.is_available():
                return torch.cuda.current_stream().cuda_stream
        except ImportError:
            pass
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _check_unpack(packed, outs, width, height, shard_count, shard_stride_tiles, packed_tile_bytes, out_bpp, what):
    # shard k's tiles start at k * shard_stride_tiles: the last shard's block ends the buffer's use
    last = shard_tile_count(width, height, shard_count - 1, shard_count) if shard_count >= 1 else 0
    _check_size(packed, ((shard_count - 1) * shard_stride_tiles + last) * packed_tile_bytes, "packed", what)
    for t, name in outs:
        _check_size(t, width * height * out_bpp, name, what)


def tiles_unpack(packed, out, width: int, height: int, shard_count: int, shard_stride_tiles: int,
                 bytes_per_pixel: int, stream=None) -> None:
    _check_unpack(packed, [(out, "out")], width, height, shard_count, shard_stride_tiles, 64 * bytes_per_pixel,
                  bytes_per_pixel, "tiles_unpack")
    check(load().bh_tiles_unpack(_ptr(packed), _ptr(out), width, height, shard_count, shard_stride_tiles,
                                 bytes_per_pixel, _stream_handle(stream)), "bh_tiles_unpack")


def tiles_unpack_rgb(packed, out, width: int, height: int, shard_count: int, shard_stride_tiles: int,
                     fmt: int, stream=None, rows_in_flight: int = 0) -> None:
    """bh_tiles_unpack_rgb(_rows): gathered BH_LAYOUT_TILES_RGB shards of format `fmt` -> row-major
    frame; rows_in_flight > 0 throttles it for overlap with a render (include/bh_render.h)."""
    bpp = _abi.BYTES_PER_PIXEL.get(fmt, 0)
    _check_unpack(packed, [(out, "out")], width, height, shard_count, shard_stride_tiles, 48 * bpp, bpp,
                  "tiles_unpack_rgb")
    if rows_in_flight:
        check(load().bh_tiles_unpack_rgb_rows(_ptr(packed), _ptr(out), width, height, shard_count,
                                              shard_stride_tiles, fmt, rows_in_flight, _stream_handle(stream)),
              "bh_tiles_unpack_rgb_rows")
    else:
        check(load().bh_tiles_unpack_rgb(_ptr(packed), _ptr(out), width, height, shard_count, shard_stride_tiles,
                                         fmt, _stream_handle(stream)), "bh_tiles_unpack_rgb")


def _rgbm_format(fmt: int):
    """(bytes per pixel of the unpacked targets, packed layout) of an RGBM unpack format (0 bytes if invalid)."""
    lay = BH_LAYOUT_TILES_RGBM14 if fmt & BH_UNPACK_RGBM14 else BH_LAYOUT_TILES_RGBM
    base = fmt & 0xFF
    ok = fmt & ~(0xFF | BH_UNPACK_RGBM14) == 0 and (lay == BH_LAYOUT_TILES_RGBM or base == BH_OUT_RGBA16F)
    return (_abi.BYTES_PER_PIXEL.get(base, 0) if ok else 0), lay


def tiles_unpack_rgbm(packed, out_col, out_blackout, width: int, height: int, shard_count: int,
                      shard_stride_tiles: int, fmt: int, stream=None, rows_in_flight: int = 0) -> None:
    """bh_tiles_unpack_rgbm: gathered BH_LAYOUT_TILES_RGBM shards -> both Scene::render targets, row-major
    (`out_blackout` None == Option::None).  fmt = BH_OUT_RGBA16F | BH_UNPACK_RGBM14: BH_LAYOUT_TILES_RGBM14
    shards."""
    bpp, lay = _rgbm_format(fmt)
    _check_unpack(packed, [(out_col, "out_col"), (out_blackout, "out_blackout")], width, height, shard_count,
                  shard_stride_tiles, tile_bytes(lay, fmt & 0xFF) if bpp else 0, bpp, "tiles_unpack_rgbm")
    check(load().bh_tiles_unpack_rgbm(_ptr(packed), _ptr(out_col), _ptr(out_blackout), width, height, shard_count,
                                      shard_stride_tiles, fmt, rows_in_flight, _stream_handle(stream)),
          "bh_tiles_unpack_rgbm")


class Partition:
    """bh_partition (include/bh_render.h): a weighted tile partition of a width x height frame over
    shard_count shards -- shard k owns weights[k] of every sum(weights) residues of (tx + 3*ty), each
    shard's packed order row-major over its tiles.  Pass it to Scene.render / render_frames
    (layout BH_LAYOUT_TILES*) and to tiles_unpack_rgbm."""

    def __init__(self, width: int, height: int, weights, device: int = 0) -> None:
        self.width, self.height = width, height
        self.weights = [int(w) for w in weights]
        self.shard_count = len(self.weights)
        w = (C.c_uint32 * self.shard_count)(*self.weights)
        h = C.c_void_p()
        check(load().bh_partition_create(width, height, self.shard_count, w, device, C.byref(h)), "bh_partition_create")
        self.handle = h.value
        self.counts = [self.tile_count(k) for k in range(self.shard_count)]

    def tile_count(self, shard_index: int) -> int:
        n = load().bh_partition_tile_count(self.handle, shard_index)
        if n < 0:
            raise BhError(int(n), "bh_partition_tile_count")
        return int(n)

    def close(self) -> None:
        if getattr(self, "handle", None):
            load().bh_partition_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def partition_map(width: int, height: int, weights):
    """bh_partition_map (host only): (owner, index) per tile t = ty * tiles_x + tx, as numpy arrays."""
    tiles = ((width + 7) // 8) * ((height + 7) // 8)
    owner = np.zeros(tiles, np.uint32)
    index = np.zeros(tiles, np.uint32)
    w = (C.c_uint32 * len(weights))(*[int(x) for x in weights])
    check(load().bh_partition_map(width, height, len(weights), w, owner.ctypes.data, index.ctypes.data),
          "bh_partition_map")
    return owner, index


def tiles_unpack_rgbm_partition(packed, out_col, out_blackout, partition: "Partition", shard_stride_tiles: int,
                                fmt: int, stream=None, rows_in_flight: int = 0) -> None:
    """bh_tiles_unpack_rgbm_partition: gathered BH_LAYOUT_TILES_RGBM shards of `partition` -> both targets
    (fmt with BH_UNPACK_RGBM14: BH_LAYOUT_TILES_RGBM14 shards)."""
    bpp, lay = _rgbm_format(fmt)
    S = partition.shard_count
    _check_size(packed, ((S - 1) * shard_stride_tiles + partition.counts[-1]) * (tile_bytes(lay, fmt & 0xFF)
                                                                                if bpp else 0), "packed",
                "tiles_unpack_rgbm_partition")
    for t, name in ((out_col, "out_col"), (out_blackout, "out_blackout")):
        _check_size(t, partition.width * partition.height * bpp, name, "tiles_unpack_rgbm_partition")
    check(load().bh_tiles_unpack_rgbm_partition(_ptr(packed), _ptr(out_col), _ptr(out_blackout), partition.handle,
                                                shard_stride_tiles, fmt, rows_in_flight, _stream_handle(stream)),
          "bh_tiles_unpack_rgbm_partition")


__all__ = ["Camera", "Partition", "Presenter", "partition_map", "tiles_unpack_rgbm_partition", "CameraController", "CameraUniform", "Uniforms", "Scene", "synthetic_sky", "shard_tile_count", "tiles_unpack",
           "tiles_unpack_rgb", "tiles_unpack_rgbm", "tile_bytes", "BH_LAYOUT_TILES_RGBM", "BH_LAYOUT_TILES_RGBM14",
           "BH_UNPACK_RGBM14",
           "srgb_encode_table", "load_sky", "bloom_plan_failures", "BH_OUT_BGRA8_SRGB",
           "BhError", "MAX_ITERATIONS", "BH_OUT_RGBA32F", "BH_OUT_RGBA16F", "BH_MATH_EXACT", "BH_MATH_FAST",
           "BH_LAYOUT_ROWMAJOR", "BH_LAYOUT_TILES", "BH_LAYOUT_TILES_RGB", "BH_SCENE_DEFAULT", "BYTES_PER_PIXEL"]
