"""CPU checks of the post-processing oracle (Kawase bloom + remix):
oracle/bh_bloom_oracle.c against the independent numpy restatement oracle/bloom_np.py, and
size-independent properties of the chain."""
import numpy as np
import pytest

import oracle
from oracle import bloom_np, oracle_np


def _img(rng, H, W, sparse=False):
    t = rng.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
    if sparse:  # mostly black with bright points: the blackout target's typical content
        t[..., :3] = np.where(rng.random((H, W, 1)) < 0.05, t[..., :3], 0)
    t[..., 3] = 255
    return t


@pytest.mark.parametrize("H,W,levels", [(16, 24, 3), (32, 32, 3), (13, 21, 2), (9, 7, 1), (40, 64, 4)])
def test_bloom_oracle_matches_numpy_restatement(H, W, levels):
    rng = np.random.default_rng(H * 1000 + W * 10 + levels)
    col, bo = _img(rng, H, W), _img(rng, H, W, sparse=True)
    a = oracle.bloom(col, bo, levels)
    b = bloom_np.bloom(col, bo, levels)
    assert np.array_equal(a, b), np.argwhere(a != b)[:5]


def test_bloom_of_constant_images_is_the_scalar_chain():
    """Every pass of a constant image is that constant (bilinear / 8-tap weights sum to 1), so the
    surface is col + 0.5 q(Y + 0.5 q(Y)) with Y = q(X + 0.5 q(X)), quantised like the stores."""
    lut = oracle_np.srgb_lut()
    for kx, kc in [(0, 0), (255, 0), (40, 200), (128, 128), (7, 250)]:
        X = np.full((24, 40, 4), [kx, kx, kx, 255], np.uint8)
        Cc = np.full((24, 40, 4), [kc, kc, kc, 255], np.uint8)
        out = oracle.bloom(Cc, X, 3)
        q = lambda v: lut[oracle.srgb_encode(np.array([v], np.float32))[0]]  # noqa: E731
        x = lut[kx]
        y = q(np.float32(x) + np.float32(q(x)) * np.float32(0.5))
        z = q(np.float32(y) + np.float32(q(y)) * np.float32(0.5))
        f = oracle.srgb_encode(np.array([np.float32(lut[kc]) + np.float32(z) * np.float32(0.5)], np.float32))[0]
        assert (out[..., :3] == f).all() and (out[..., 3] == 255).all(), (kx, kc, out[0, 0], f)


def test_bloom_spreads_a_point_and_keeps_col():
    """A single bright blackout texel glows into its neighbourhood; with a black blackout target the
    surface is exactly col (every remix adds 0.5 * 0)."""
    W, H = 64, 32
    col = _img(np.random.default_rng(3), H, W)
    bo = np.zeros((H, W, 4), np.uint8)
    bo[..., 3] = 255
    assert np.array_equal(oracle.bloom(col, bo, 3), col)
    bo[16, 32, :3] = 255
    out = oracle.bloom(np.zeros_like(col) + np.array([0, 0, 0, 255], np.uint8), bo, 3)
    lit = out[..., :3].max(-1) > 0
    ys, xs = np.nonzero(lit)
    assert lit.sum() > 9 and ys.min() < 16 < ys.max() and xs.min() < 32 < xs.max()


BLOOM_GOLDEN = sorted((__import__("pathlib").Path(__file__).parent / "golden").glob("bloom_*.npz"))


@pytest.mark.parametrize("path", BLOOM_GOLDEN, ids=[p.stem for p in BLOOM_GOLDEN])
def test_bloom_oracle_reproduces_golden(path):
    z = np.load(path)
    assert np.array_equal(oracle.bloom(z["col"], z["blackout"], int(z["levels"][0])), z["out"])
