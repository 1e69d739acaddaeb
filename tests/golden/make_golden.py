"""Generate the committed golden fixtures tests/golden/*.npz.

PARITY UNPINNED: the reference (Rust + WGSL on wgpu) cannot run in this environment and ships no
tests, vectors or fixtures, so these fixtures are outputs of OUR CPU oracle
(oracle/bh_oracle.c), each one cross-checked bit-for-bit at generation time against the independent
numpy restatement (oracle/oracle_np.py).  They pin the oracle and the GPU kernel against
regressions and against each other; they are not reference outputs.

Each fixture holds its inputs (112-byte camera uniform, 32-byte uniforms, a small RGBA8 sky, frame
size, RK cap, scene flags) and expected outputs (col RGBA f32, n_rk u16, fate u8).

bloom_*.npz: the post-processing chain (oracle/bh_bloom_oracle.c, cross-checked against
oracle/bloom_np.py): inputs col / blackout BGRA8 + levels, expected surface BGRA8.

    python tests/golden/make_golden.py [--only march|bloom]
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))

import black_hole_ray_marching_amd as bh  # noqa: E402  (camera/uniform packing + sky generator)
import oracle  # noqa: E402
from oracle import oracle_np  # noqa: E402
from tests._cases import camera_uniform, uniforms  # noqa: E402

FIXTURES = {
    # name: (camera, W, H, cap, flags, uniform overrides)
    "camA_64x32_cap512": ("A", 64, 32, 512, 3, {}),
    "camA_48x48_cap64_nodisc": ("A", 48, 48, 64, 0, {}),          # BASELINE config 1 (reduced size)
    "camB_64x36_cap256": ("B", 64, 36, 256, 3, {}),               # BASELINE config 2 camera / cap
    "camC_56x40_cap1000": ("C", 56, 40, 1000, 3, {}),             # BASELINE config 5 camera / cap
    "camD_40x24_cap512_noblackout": ("D", 40, 24, 512, 3, {"blackout_eh": 0}),
    "camB_40x24_cap512_dp0": ("B", 40, 24, 512, 3, {"distortion_power": 0.0}),
    "camE_48x32_cap512_zeno": ("E", 48, 32, 512, 3, {}),           # shadow edge: capped rays
    "camE_40x24_cap1000_zeno": ("E", 40, 24, 1000, 3, {}),
}
SKY_W, SKY_H, SKY_SEED = 128, 64, 0x5EED_B1AC_401E


def make(name, spec, sky):
    cam, W, H, cap, flags, over = spec
    cu, U = camera_uniform(cam, W, H), uniforms(**over)
    col, _, n_rk, fate = oracle.render_rows(cu.to_bytes(), bytes(U.to_c()), sky, W, H, cap, flags)
    with np.errstate(all="ignore"):
        c2, _, n2, f2 = oracle_np.render(cu.pos, cu.world_tri, U.as_dict(), sky, W, H, cap, flags)
    assert np.array_equal(col.view(np.uint32), c2.view(np.uint32)), name
    assert np.array_equal(n_rk, n2) and np.array_equal(fate, f2), name
    np.savez_compressed(HERE / f"{name}.npz", camera_uniform=np.frombuffer(cu.to_bytes(), np.uint8),
                        uniforms=np.frombuffer(bytes(U.to_c()), np.uint8), sky=sky,
                        meta=np.array([W, H, cap, flags], np.uint32), col=col, n_rk=n_rk, fate=fate)
    print(name, np.bincount(fate.ravel(), minlength=4), float(n_rk.mean()))


def _bgra(c):
    e = oracle.srgb_encode(c[..., :3])
    return np.stack([e[..., 2], e[..., 1], e[..., 0], np.full(e.shape[:2], 255, np.uint8)], -1)


def make_bloom(sky):
    from oracle import bloom_np
    cu, U = camera_uniform("A", 64, 32), uniforms()
    col, bo, _, _ = oracle.render_rows(cu.to_bytes(), bytes(U.to_c()), sky, 64, 32, 512, 3)
    rng = np.random.default_rng(0xB100)
    rnd = rng.integers(0, 256, size=(30, 50, 4), dtype=np.uint8)
    rnd[..., 3] = 255
    sparse = rnd.copy()
    sparse[..., :3] = np.where(rng.random((30, 50, 1)) < 0.05, sparse[..., :3], 0)
    cases = {"bloom_camA_64x32_l3": (_bgra(col), _bgra(bo), 3),
             "bloom_random_50x30_l2": (rnd, sparse, 2),
             "bloom_random_32x30_l1": (rnd[:, :32].copy(), sparse[:, :32].copy(), 1)}
    for name, (c, b, lv) in cases.items():
        out = oracle.bloom(c, b, lv)
        assert np.array_equal(out, bloom_np.bloom(c, b, lv)), name
        np.savez_compressed(HERE / f"{name}.npz", col=c, blackout=b, levels=np.array([lv], np.uint32), out=out)
        print(name, out.shape, float(out[..., :3].mean()))


def main():
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    sky = bh.synthetic_sky(SKY_W, SKY_H, SKY_SEED)
    if only in (None, "march"):
        for name, spec in FIXTURES.items():
            make(name, spec, sky)
    if only in (None, "bloom"):
        make_bloom(sky)


if __name__ == "__main__":
    main()
