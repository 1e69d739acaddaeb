"""TEST INFRASTRUCTURE: an independent numpy restatement of the reference's Kawase bloom + remix chain
(src/bloom.rs:53-71, src/blur.rs:37-45, src/kawase_downsampling.rs:250-306,
src/kawase_upsampling.rs:192-210,241-295, src/kawase_downsample.wgsl:23-36,
src/kawase_upsample.wgsl:23-38, src/remix.wgsl:20-25, src/copy.wgsl:15-19), written separately from
oracle/bh_bloom_oracle.c from the same lines, vectorised per pass; small images only.  PARITY
UNPINNED (see bh_bloom_oracle.c): the normative sampler and store are restated there."""
from __future__ import annotations

import numpy as np

from .oracle_np import srgb_lut

f32 = np.float32


def _encode(x: np.ndarray) -> np.ndarray:
    """Normative Bgra8UnormSrgb store of linear values (oracle bho_srgb_encode), element-wise."""
    v = x.astype(np.float64)
    s = np.where(v <= 0.0031308, 12.92 * v, 1.055 * np.power(np.maximum(v, 0.0), 1.0 / 2.4) - 0.055)
    q = np.floor(s * 255.0 + 0.5)
    q = np.where(~(x > 0), 0.0, np.where(x >= 1, 255.0, np.minimum(q, 255.0)))
    return q.astype(np.uint8)


def _unorm(a: np.ndarray) -> np.ndarray:
    q = np.floor(a.astype(np.float64) * 255.0 + 0.5)
    return np.where(~(a > 0), 0.0, np.where(a >= 1, 255.0, q)).astype(np.uint8)


def _decode(t: np.ndarray) -> np.ndarray:
    """(h, w, 4) BGRA8 -> (h, w, 4) linear RGBA f32."""
    lut = srgb_lut()
    return np.stack([lut[t[..., 2]], lut[t[..., 1]], lut[t[..., 0]], t[..., 3].astype(f32) / f32(255)], -1)


def _store(c: np.ndarray) -> np.ndarray:
    return np.stack([_encode(c[..., 2]), _encode(c[..., 1]), _encode(c[..., 0]), _unorm(c[..., 3])], -1)


def _sample(tex: np.ndarray, u: np.ndarray, v: np.ndarray) -> np.ndarray:
    """Clamp-to-edge bilinear (f32 weights, lerp x then y) of a BGRA8 texture at texcoords u, v."""
    h, w = tex.shape[:2]
    d = _decode(tex)
    tx = np.minimum(np.maximum(u * f32(w) - f32(0.5), f32(-1)), f32(w))
    ty = np.minimum(np.maximum(v * f32(h) - f32(0.5), f32(-1)), f32(h))
    fx, fy = np.floor(tx), np.floor(ty)
    fa, fb = (tx - fx)[..., None], (ty - fy)[..., None]
    x0, y0 = fx.astype(np.int64), fy.astype(np.int64)
    x1, y1 = np.clip(x0 + 1, 0, w - 1), np.clip(y0 + 1, 0, h - 1)
    x0, y0 = np.clip(x0, 0, w - 1), np.clip(y0, 0, h - 1)
    ia, ib = f32(1) - fa, f32(1) - fb
    top = d[y0, x0] * ia + d[y0, x1] * fa
    bot = d[y1, x0] * ia + d[y1, x1] * fa
    return (top * ib + bot * fb).astype(f32)


def _uv(w: int, h: int):
    u = (np.arange(w, dtype=f32) + f32(0.5)) / f32(w)
    v = (np.arange(h, dtype=f32) + f32(0.5)) / f32(h)
    return np.meshgrid(u, v)


def _pass(kind: str, a: np.ndarray, out_wh, res=None, b: np.ndarray | None = None) -> np.ndarray:
    w, h = out_wh
    U, V = _uv(w, h)
    if kind in ("copy", "down"):
        c = _sample(a, U, V)
    elif kind == "up":
        hx, hy = f32(0.5) / f32(res[0]), f32(0.5) / f32(res[1])
        o = f32(3)
        taps = [((-hx * f32(2)) * o, f32(0) * o, 1), ((-hx) * o, hy * o, 2), (f32(0) * o, (hy * f32(2)) * o, 1),
                (hx * o, hy * o, 2), ((hx * f32(2)) * o, f32(0) * o, 1), (hx * o, (-hy) * o, 2),
                (f32(0) * o, (-hy * f32(2)) * o, 1), ((-hx) * o, (-hy) * o, 2)]
        c = None
        for du, dv, wgt in taps:
            t = _sample(a, U + du, V + dv)
            t = t * f32(2) if wgt == 2 else t
            c = t if c is None else c + t
        c = c / f32(12)
    else:  # remix
        c = _sample(a, U, V) + _sample(b, U, V) * f32(0.5)
    return _store(c)


def _resolutions(W: int, H: int, levels: int):
    out, w, h = [], W, H
    for _ in range(levels):
        w, h = max(w, 1), max(h, 1)
        out.append((w, h))
        w, h = w // 2, h // 2
    return out


def _blur(inp: np.ndarray, levels: int) -> np.ndarray:
    H, W = inp.shape[:2]
    res = _resolutions(W, H, levels)
    down = [inp] + [None] * (levels - 1)
    for lv in range(1, levels):
        down[lv] = _pass("down", down[lv - 1], res[lv])
    up = [None] * levels
    up[levels - 1] = _pass("down", down[levels - 1], res[levels - 1])
    for lv in range(levels - 1):
        up[levels - lv - 2] = _pass("up", up[levels - lv - 1], res[levels - lv - 2], res[lv])
    return _pass("up", up[0], (W, H), res[levels - 1])


def bloom(col: np.ndarray, blackout: np.ndarray, levels: int = 3) -> np.ndarray:
    """Bloom::render: (H, W, 4) BGRA8 col and blackout -> the surface (H, W, 4) BGRA8."""
    H, W = col.shape[:2]
    copies = [blackout] + [None] * (levels - 1)
    for level in range(levels - 1):
        blur_in = _pass("copy", copies[0], (W, H))
        r0 = _pass("copy", copies[0], (W, H))
        r1 = _blur(blur_in, 1)
        copies[level + 1] = _pass("remix", r0, (W, H), b=r1)
    L = levels - 1
    blur_in = _pass("copy", copies[L], (W, H))
    r0 = _pass("copy", copies[L], (W, H))
    r1 = _blur(blur_in, levels)
    final_in1 = _pass("remix", r0, (W, H), b=r1)
    return _pass("remix", col, (W, H), b=final_in1)
