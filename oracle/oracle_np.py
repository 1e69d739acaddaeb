"""Independent numpy restatement of the hot path.  TEST INFRASTRUCTURE ONLY.

Used in this container to cross-check the C oracle (oracle/bh_oracle.c) — the two are written
separately from src/black_hole_maybe.wgsl and must agree bit-for-bit, because both follow the same
normative arithmetic (oracle/bh_oracle.c header; DESIGN.md "Normative arithmetic"): numpy float32
ops are IEEE single precision with no FMA contraction, exactly like the C oracle built with
-ffp-contract=off.  Vectorised over pixels; intended for frames up to ~256x256.

PARITY UNPINNED (no reference fixtures exist; the reference cannot run here) — see SURVEY.md §8c.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32

FATE_CAP, FATE_ESCAPE, FATE_SURFACE, FATE_BLACKOUT = 0, 1, 2, 3
SCENE_DISC, SCENE_MARKERS = 1, 2

MIN_DIST = f32(0.001)          # src/black_hole_maybe.wgsl:80
TWO_PI = f32(6.28318530718)    # :82
ONE_PI = f32(3.14159265359)    # :83


def _dot(ax, ay, az, bx, by, bz):
    return (ax * bx + ay * by) + az * bz


def _len(x, y, z):
    return np.sqrt(_dot(x, y, z, x, y, z))


def _pow25(q):  # pow(q, 2.5) := (q*q)*sqrt(q) in f32 (normative)
    return (q * q) * np.sqrt(q)


def _pow15(c):  # pow(c, 1.5) := c*sqrt(c) in f32
    return c * np.sqrt(c)


def srgb_lut():
    c = np.arange(256, dtype=np.float64) / 255.0
    return np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4).astype(f32)


def _sdf_sphere(px, py, pz, cx, cy, cz, r):  # :91-93  length(centre - p) - r
    return _len(f32(cx) - px, f32(cy) - py, f32(cz) - pz) - f32(r)


def _sdf(px, py, pz, rs, flags):  # :95-123
    d = np.full(px.shape, np.inf, dtype=f32)
    if flags & SCENE_DISC:
        rho = np.sqrt(px * px + pz * pz)
        a = rho - f32(6.0) * rs
        b = -(rho - f32(3.0) * rs)
        plane = np.abs(py - f32(0.0)) - f32(0.02)
        d = np.fmax(np.fmax(a, b), plane)
    if flags & SCENE_MARKERS:
        s1 = _sdf_sphere(px, py, pz, 0.0, 10.0, -10.0, 0.5)
        s2 = _sdf_sphere(px, py, pz, 0.0, -10.0, -10.0, 0.5)
        s3 = _sdf_sphere(px, py, pz, 10.0, 0.0, -10.0, 0.5)
        s4 = _sdf_sphere(px, py, pz, -10.0, 0.0, -10.0, 0.5)
        m = np.fmin(s1, np.fmin(s2, np.fmin(s3, s4)))
        d = np.fmin(d, m) if flags & SCENE_DISC else m
    return d


def _accel(s, x, y, z):  # :125-127  (s * ro) / pow(dot(ro,ro), 2.5), s = ((DP*RS)*-1.5)*h2
    p = _pow25(_dot(x, y, z, x, y, z))
    return (s * x) / p, (s * y) / p, (s * z) / p


def _sample(sky, lut, u, v):
    h, w = sky.shape[0], sky.shape[1]
    nan = np.isnan(u) | np.isnan(v)
    u = np.where(nan, f32(0), u)
    v = np.where(nan, f32(0), v)
    tx = u * f32(w) - f32(0.5)
    ty = v * f32(h) - f32(0.5)
    tx = np.fmin(np.fmax(tx, f32(-1)), f32(w))
    ty = np.fmin(np.fmax(ty, f32(-1)), f32(h))
    fx, fy = np.floor(tx), np.floor(ty)
    a, b = tx - fx, ty - fy
    x0, y0 = fx.astype(np.int64), fy.astype(np.int64)
    x1, y1 = np.clip(x0 + 1, 0, w - 1), np.clip(y0 + 1, 0, h - 1)
    x0, y0 = np.clip(x0, 0, w - 1), np.clip(y0, 0, h - 1)
    ia, ib = f32(1) - a, f32(1) - b
    out = []
    for ch in range(3):
        t = lut[sky[:, :, ch]]
        t00, t10, t01, t11 = t[y0, x0], t[y0, x1], t[y1, x0], t[y1, x1]
        top = t00 * ia + t10 * a
        bot = t01 * ia + t11 * a
        c = top * ib + bot * b
        c = np.where(nan, t[0, 0], c)
        out.append(c.astype(f32))
    return out


def get_col(ro0, rd0, U, sky, max_iters, flags):
    """Vectorised get_col (src/black_hole_maybe.wgsl:259-345).

    ro0: (3,) float32 camera position; rd0: (N,3) float32 unit directions.
    U: dict with rs, delta_time_mult, blackout_eh, max_dist, distortion_power.
    Returns (rgb (N,3) f32, n_rk (N,) int, fate (N,) int).
    """
    n = rd0.shape[0]
    rs, dtm = f32(U["rs"]), f32(U["delta_time_mult"])
    maxd, dp = f32(U["max_dist"]), f32(U["distortion_power"])
    blackout = int(U["blackout_eh"]) != 0
    rox = np.full(n, ro0[0], f32); roy = np.full(n, ro0[1], f32); roz = np.full(n, ro0[2], f32)
    rdx, rdy, rdz = rd0[:, 0].copy(), rd0[:, 1].copy(), rd0[:, 2].copy()
    cx = roy * rdz - roz * rdy; cy = roz * rdx - rox * rdz; cz = rox * rdy - roy * rdx  # :262
    h2 = _dot(cx, cy, cz, cx, cy, cz)                                                 # :263
    s = ((dp * rs) * f32(-1.5)) * h2
    ln = _len(f32(ro0[0]), f32(ro0[1]), f32(ro0[2]))
    nx, ny, nz = f32(ro0[0]) / ln, f32(ro0[1]) / ln, f32(ro0[2]) / ln
    cpx, cpy, cpz = (-nx * f32(1.5)) * rs, (-ny * f32(1.5)) * rs, (-nz * f32(1.5)) * rs  # :294
    travelled = np.zeros(n, f32)
    outside = np.zeros(n, bool)
    alive = np.ones(n, bool)
    n_rk = np.zeros(n, np.int64)
    fate = np.full(n, FATE_CAP, np.int64)
    rgb = np.zeros((n, 3), f32)
    for _ in range(max_iters):                                                         # :266
        if not alive.any():
            break
        r = _len(rox, roy, roz)                                                        # :271
        if blackout:                                                                   # :272-283
            hit = alive & (r < f32(1)) & (_dot(rdx, rdy, rdz, rox, roy, roz) < f32(0))
            fate[hit] = FATE_BLACKOUT; alive &= ~hit
            outside |= alive & (r > f32(1))
            hit = alive & ~(r > f32(1)) & outside
            fate[hit] = FATE_BLACKOUT; alive &= ~hit
        ds = _sdf(rox, roy, roz, rs, flags)                                            # :285
        hit = alive & (ds < MIN_DIST)                                                  # :286
        fate[hit] = FATE_SURFACE; rgb[hit] = 1.0; alive &= ~hit
        dps = _sdf_sphere(rox, roy, roz, cpx, cpy, cpz, 0.075)                         # :294
        dist = np.fmin(ds, dps)
        dd = np.fmin(dist * f32(0.9), dtm * r)                                      # :307-310
        dt = dd
        # get_delta_photon_rk4 (:134-151)
        a1 = _accel(s, rox, roy, roz)
        rok1 = (dt * rdx, dt * rdy, dt * rdz)
        rdk1 = (dt * a1[0], dt * a1[1], dt * a1[2])
        rok2 = tuple(dt * (v + f32(0.5) * k) for v, k in zip((rdx, rdy, rdz), rdk1))
        a2 = _accel(s, *(p + f32(0.5) * k for p, k in zip((rox, roy, roz), rok1)))
        rdk2 = tuple(dt * a for a in a2)
        rok3 = tuple(dt * (v + f32(0.5) * k) for v, k in zip((rdx, rdy, rdz), rdk2))
        a3 = _accel(s, *(p + f32(0.5) * k for p, k in zip((rox, roy, roz), rok2)))
        rdk3 = tuple(dt * a for a in a3)
        rok4 = tuple(dt * (v + k) for v, k in zip((rdx, rdy, rdz), rdk3))
        a4 = _accel(s, *(p + k for p, k in zip((rox, roy, roz), rok3)))
        rdk4 = tuple(dt * a for a in a4)
        dro = [(((k1 + f32(2) * k2) + f32(2) * k3) + k4) / f32(6) for k1, k2, k3, k4 in zip(rok1, rok2, rok3, rok4)]
        drd = [(((k1 + f32(2) * k2) + f32(2) * k3) + k4) / f32(6) for k1, k2, k3, k4 in zip(rdk1, rdk2, rdk3, rdk4)]
        rox = np.where(alive, rox + dro[0], rox); roy = np.where(alive, roy + dro[1], roy)
        roz = np.where(alive, roz + dro[2], roz)
        rdx = np.where(alive, rdx + drd[0], rdx); rdy = np.where(alive, rdy + drd[1], rdy)
        rdz = np.where(alive, rdz + drd[2], rdz)
        travelled = np.where(alive, travelled + dd, travelled)
        n_rk += alive
        esc = alive & (travelled > maxd)                                               # :325
        fate[esc] = FATE_ESCAPE; alive &= ~esc
    sky_rays = (fate == FATE_CAP) | (fate == FATE_ESCAPE)
    ln = _len(rdx, rdy, rdz)                                                           # :330
    nx, ny, nz = rdx / ln, rdy / ln, rdz / ln
    az = np.arctan2(nz.astype(np.float64), nx.astype(np.float64)).astype(f32)          # :332
    x = (az + ONE_PI) / TWO_PI                                                         # :334
    y = (ny + f32(1)) * f32(0.5)                                                       # :336
    lut = srgb_lut()
    r_, g_, b_ = _sample(sky, lut, x, f32(1) - y)                                      # :341
    g_, b_ = _pow15(g_), _pow15(b_)                                                    # :342-343
    rgb[sky_rays, 0] = r_[sky_rays]; rgb[sky_rays, 1] = g_[sky_rays]; rgb[sky_rays, 2] = b_[sky_rays]
    return rgb, n_rk, fate


def pixel_dirs(cam_world_tri, width, height):
    """Interpolated, normalised per-pixel ray directions (vs_main + rasteriser, :37-55, :362)."""
    px = np.arange(width, dtype=f32)
    py = np.arange(height, dtype=f32)
    l0 = (px + f32(0.5)) / (f32(2) * f32(width))
    l2 = (py + f32(0.5)) / (f32(2) * f32(height))
    L0, L2 = np.meshgrid(l0, l2)
    L1 = (f32(1) - L0) - L2
    c = np.asarray(cam_world_tri, dtype=f32)
    d = [((L0 * c[0, k] + L1 * c[1, k]) + L2 * c[2, k]).ravel() for k in range(3)]
    ln = _len(*d)
    return np.stack([d[0] / ln, d[1] / ln, d[2] / ln], axis=1)


def render(cam_pos, cam_world_tri, U, sky, width, height, max_iters, flags):
    """Full frame: returns col (H,W,4), blackout (H,W,4), n_rk (H,W), fate (H,W)."""
    rd0 = pixel_dirs(cam_world_tri, width, height)
    rgb, n_rk, fate = get_col(np.asarray(cam_pos, f32), rd0, U, sky, max_iters, flags)
    col = np.concatenate([rgb, np.ones((rgb.shape[0], 1), f32)], axis=1)
    keep = ~(_dot(rgb[:, 0], rgb[:, 1], rgb[:, 2], rgb[:, 0], rgb[:, 1], rgb[:, 2]) < f32(1))  # :366
    bo = np.where(keep[:, None], col, np.array([0, 0, 0, 1], f32))
    shape = (height, width)
    return (col.reshape(*shape, 4), bo.reshape(*shape, 4).astype(f32),
            n_rk.reshape(shape), fate.reshape(shape))
