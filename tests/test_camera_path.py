"""CameraController (src/camera.rs:115-366) through the C ABI against an independent numpy f32
restatement of update_camera (glam 0.24 Quat::from_axis_angle / mul_vec3; f32 sin/cos/exp from the
platform libm, which Rust's f32 methods call too).  Parity: bit-exact over random key sequences.
glam is not vendored in the reference (Cargo.lock:722-723): the Quat formulas are restated from its
published source, so this pins the C++ against the restatement, not against glam itself."""
import ctypes as C
import ctypes.util

import numpy as np
import pytest

import black_hole_ray_marching_amd as bh

f32 = np.float32
_m = C.CDLL(ctypes.util.find_library("m"))
for _n in ("sinf", "cosf", "expf"):
    getattr(_m, _n).restype = C.c_float
    getattr(_m, _n).argtypes = [C.c_float]


def _sinf(x): return f32(_m.sinf(float(x)))  # noqa: E704
def _cosf(x): return f32(_m.cosf(float(x)))  # noqa: E704
def _expf(x): return f32(_m.expf(float(x)))  # noqa: E704


def dot(a, b): return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]  # noqa: E704


def cross(a, b):
    return np.array([a[1] * b[2] - b[1] * a[2], a[2] * b[0] - b[2] * a[0], a[0] * b[1] - b[0] * a[1]], f32)


def quat(axis, angle):
    h = f32(angle) * f32(0.5)
    s, c = _sinf(h), _cosf(h)
    return np.array([axis[0] * s, axis[1] * s, axis[2] * s], f32), c


def qmul(q, v):
    b, w = q
    return (v * (w * w - dot(b, b)) + b * (dot(v, b) * f32(2))) + cross(b, v) * (w * f32(2))


def norm(neg, pos):
    return f32(0) if neg == pos else (f32(1) if pos else f32(-1))


def update(st, pos, dir_, up, dt, do_pan):
    dt = f32(dt)
    right = lambda: cross(up, dir_)  # noqa: E731
    xn, zn, yn = norm(st["left"], st["right"]), norm(st["backward"], st["forward"]), norm(st["down"], st["up"])
    sp = f32(st["speed"])
    pos = pos + right() * ((dt * sp) * xn)
    pos = pos + dir_ * ((dt * sp) * zn)
    pos = pos + up * ((dt * sp) * yn)
    pos = pos * _expf(-dt * norm(st["exp_towards_origin"], st["exp_away_origin"]))
    ps = f32(st["pan_speed"])
    xpn, ypn = norm(st["pan_left"], st["pan_right"]), norm(st["pan_up"], st["pan_down"])
    for axis_fn, ang in ((lambda: np.array([0, 1, 0], f32), (dt * ps) * xpn), (right, (dt * ps) * ypn)):
        q = quat(axis_fn(), ang)
        dir_, up = qmul(q, dir_), qmul(q, up)
    if st["mouse_pressed"] and do_pan:
        # cursor_movement (:268-278): zero until two positions are known
        m = np.array(st["curr"], f32) - np.array(st["prev"], f32) if st["prev"] is not None else np.zeros(2, f32)
        for axis_fn, ang in ((lambda: np.array([0, 1, 0], f32), (dt * ps) * m[0]), (right, (dt * ps) * m[1])):
            q = quat(axis_fn(), ang)
            dir_, up = qmul(q, dir_), qmul(q, up)
    return pos.astype(f32), dir_.astype(f32), up.astype(f32), bool(xn or yn or zn or xpn or ypn)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_controller_path_matches_restatement(seed):
    rng = np.random.default_rng(seed)
    k = bh.CameraController()
    cam = bh.Camera.default(4096, 2048)
    pos, dir_, up = (np.array(v, f32) for v in (cam.pos, cam.dir, cam.up))
    st = {"speed": k.c.speed, "pan_speed": k.c.pan_speed, "mouse_pressed": 0, "prev": None, "curr": None}
    for name in bh.CameraController.KEYS.values():
        st[name] = 0
    for frame in range(60):
        for key in rng.choice(list(bh.CameraController.KEYS) + ["Q", "E"], size=2):
            pressed = bool(rng.integers(0, 2))
            k.process_key(str(key), pressed)
            if key in bh.CameraController.KEYS:
                st[bh.CameraController.KEYS[key]] = int(pressed)
            elif pressed:
                st["speed"] = float(f32(st["speed"]) / f32(1.5) if key == "Q" else f32(st["speed"]) * f32(1.5))
        k.process_mouse(bool(rng.integers(0, 2)))
        st["mouse_pressed"] = k.c.mouse_pressed
        x, y = rng.uniform(0, 2000, 2)
        st["prev"], st["curr"] = st["curr"], (f32(x), f32(y))
        k.process_cursor(x, y)
        dt = float(rng.uniform(0.001, 0.05))
        do_pan = bool(rng.integers(0, 2))
        cam, moved = k.update_camera(cam, dt, do_pan)
        pos, dir_, up, moved_ref = update(st, pos, dir_, up, dt, do_pan)
        assert np.array_equal(np.array(cam.pos, f32).view(np.uint32), pos.view(np.uint32)), frame
        assert np.array_equal(np.array(cam.dir, f32).view(np.uint32), dir_.view(np.uint32)), frame
        assert np.array_equal(np.array(cam.up, f32).view(np.uint32), up.view(np.uint32)), frame
        assert moved == moved_ref


def test_controller_semantics():
    """W moves along dir by speed*dt; P ("exp towards origin") scales pos by exp(+dt) -- the
    reference's sign (camera.rs:313-323: towards -> norm -1 -> pos * exp(-dt * -1)), kept; a left
    pan turns dir about +Y."""
    k = bh.CameraController(speed=2.0)
    cam = bh.Camera.default(64, 32)
    k.process_key("W", True)
    c1, moved = k.update_camera(cam, 0.5)
    assert moved and np.allclose(c1.pos, (0, 0, -19), atol=1e-6)
    k.process_key("W", False)
    k.process_key("P", True)
    c2, moved = k.update_camera(c1, 0.5)
    assert not moved and np.isclose(np.linalg.norm(c2.pos), 19 * np.exp(0.5), rtol=1e-6)
    k.process_key("P", False)
    k.process_key("ArrowLeft", True)
    c3, _ = k.update_camera(c2, 1.0)
    assert c3.dir[0] < 0 and np.isclose(np.linalg.norm(c3.dir), 1.0, rtol=1e-5)


def test_png_roundtrip():
    from black_hole_ray_marching_amd.png import decode_png_rgba, encode_png
    rng = np.random.default_rng(0)
    bgra = rng.integers(0, 256, size=(17, 23, 4), dtype=np.uint8)
    rgba = decode_png_rgba(encode_png(bgra))
    assert np.array_equal(rgba, bgra[..., [2, 1, 0, 3]])
