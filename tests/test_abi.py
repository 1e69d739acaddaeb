"""CPU tests of the C ABI library and the host-side logic (no kernel launches: no GPU here)."""
import ctypes as C
import hashlib
import re
from pathlib import Path

import numpy as np
import pytest

import black_hole_ray_marching_amd as bh
from black_hole_ray_marching_amd import _abi, multigpu

HEADER = Path(__file__).resolve().parent.parent / "include" / "bh_render.h"


def declared_functions():
    txt = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w]+\**\s+\**(bh_\w+)\s*\(", txt, flags=re.M)))


def test_library_exports_every_declared_symbol():
    lib = bh.load()
    names = declared_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) <= set(_abi.SIGNATURES), set(names) - set(_abi.SIGNATURES)


def test_abi_version_and_status_strings():
    lib = bh.load()
    assert lib.bh_abi_version() == _abi.ABI_VERSION == 8
    # the Python mirror's constants are the header's
    text = HEADER.read_text()
    for name, value in (("BH_ABI_VERSION", _abi.ABI_VERSION), ("BH_MAX_FRAMES", _abi.BH_MAX_FRAMES),
                        ("BH_ORDER_STATES", _abi.BH_ORDER_STATES), ("BH_BLOOM_SETS", _abi.BH_BLOOM_SETS),
                        ("BH_PRESENT_BATCH_MAX", _abi.BH_PRESENT_BATCH_MAX)):
        assert re.search(rf"#define {name} {value}\b", text), name
    assert lib.bh_status_string(0) == b"ok"
    assert lib.bh_status_string(-1) == b"invalid argument"


def test_struct_layouts_match_wgsl():
    # WGSL Camera (src/black_hole_maybe.wgsl:9-17): pos @0, screen tri @16, world tri @64, 112 B
    assert C.sizeof(_abi.bh_camera_uniform) == 112
    assert _abi.bh_camera_uniform.screen_tri.offset == 16
    assert _abi.bh_camera_uniform.world_tri.offset == 64
    # WGSL Uniforms (:58-69): six 4-byte fields + vec2<u32> padding, 32 B
    assert C.sizeof(_abi.bh_uniforms) == 32
    assert _abi.bh_uniforms.blackout_eh.offset == 12 and _abi.bh_uniforms.distortion_power.offset == 20


def test_uniform_defaults_follow_scene_new():
    u = bh.Uniforms.default()  # src/scene.rs:89-137; PodBool::r#false() -> inner 1 (src/podbool.rs:24-26)
    assert (u.rs, u.delta_time_mult, u.bg_brightness, u.blackout_eh, u.max_dist, u.distortion_power) == \
        (1.0, 0.5, 0.5, 1, 250.0, 1.0)
    raw = bytes(u.to_c())
    assert raw[24:] == b"\0" * 8


def _glam_corners(pos, dir_, up, fovy, aspect):
    """Independent numpy restatement of CameraUniform::update (src/uniforms.rs:123-133,
    src/camera.rs:56-112) with an exact rigid inverse of look_at_rh."""
    f32 = np.float32
    pos, dir_, up = (np.asarray(v, f32) for v in (pos, dir_, up))

    def norm(v):
        return v * (f32(1) / np.sqrt(f32((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])))
    f = norm((pos + dir_) - pos)
    s = norm(np.array([f[1] * up[2] - up[1] * f[2], f[2] * up[0] - up[2] * f[0], f[0] * up[1] - up[0] * f[1]], f32))
    u = np.array([s[1] * f[2] - f[1] * s[2], s[2] * f[0] - f[2] * s[0], s[0] * f[1] - f[0] * s[1]], f32)
    ty = f32(np.tan(f32(fovy) / f32(2)))
    tx = ty * f32(aspect)
    out = []
    for cx, cy in ((3.0, 1.0), (-1.0, 1.0), (-1.0, -3.0)):
        dc = -np.array([tx * f32(cx), -ty * f32(cy), f32(1)], f32)
        res = s * dc[0]
        res = u * dc[1] + res
        res = (-f) * dc[2] + res
        out.append(res)
    return np.array(out, f32)


def test_default_camera_corner_rays():
    """default camera at aspect 2 -> corners (6,1,1), (-2,1,1), (-2,-3,1)."""
    cu = bh.CameraUniform()
    cu.update(bh.Camera.default(4096, 2048))
    assert np.array_equal(cu.world_tri, np.array([[6, 1, 1], [-2, 1, 1], [-2, -3, 1]], np.float32))
    assert np.array_equal(cu.pos, np.array([0, 0, -20], np.float32))
    assert [list(cu.c.screen_tri[i])[:2] for i in range(3)] == [[3, 1], [-1, 1], [-1, -3]]


@pytest.mark.parametrize("pos,target,W,H", [((0.0, 3.0, -20.0), (0.0, 0.0, 0.0), 1920, 1080),
                                            ((0.0, 6.0, -12.0), (0.0, 0.0, 0.0), 4096, 2048),
                                            ((7.0, 1.5, -9.0), (0.0, 0.0, 0.0), 640, 480)])
def test_camera_uniform_matches_numpy_restatement(pos, target, W, H):
    cam = bh.Camera.look_at(pos, target, W, H)
    cu = bh.CameraUniform()
    cu.update(cam)
    exp = _glam_corners(cam.pos, cam.dir, cam.up, cam.fovy, cam.aspect)
    assert np.array_equal(cu.world_tri, exp)


def test_synthetic_sky_is_deterministic_and_thread_count_independent():
    a = bh.synthetic_sky(512, 256)
    b = bh.synthetic_sky(512, 256)
    assert np.array_equal(a, b) and a.shape == (256, 512, 4) and np.all(a[..., 3] == 255)
    assert 10 < a[..., :3].mean() < 200
    h = hashlib.sha256(bh.synthetic_sky(4096, 2048).tobytes()).hexdigest()
    assert h.startswith("32abeface1448e9a"), h


@pytest.mark.parametrize("W,H", [(64, 64), (100, 52), (4096, 2048), (8192, 4096), (11584, 5792)])
@pytest.mark.parametrize("S", [1, 2, 3, 4, 5, 6, 8])
def test_shard_tile_counts_partition_the_frame(W, H, S):
    counts = [bh.shard_tile_count(W, H, k, S) for k in range(S)]
    assert sum(counts) == ((W + 7) // 8) * ((H + 7) // 8)
    assert counts == [multigpu.shard_tile_count(W, H, k, S) for k in range(S)]
    if W * H >= 4096 * 2048:
        assert max(counts) - min(counts) <= (H + 7) // 8  # balanced to within a tile per row


def test_shard_tiles_cover_each_tile_exactly_once():
    W, H, S = 100, 52, 5
    seen = np.zeros(((H + 7) // 8, (W + 7) // 8), int)
    for k in range(S):
        for tx, ty in multigpu.shard_tiles(W, H, k, S):
            assert (tx + 3 * ty) % S == k
            seen[ty, tx] += 1
    assert np.all(seen == 1)


def test_unpack_reference_roundtrip():
    W, H, S = 44, 30, 3
    stride = multigpu.packed_stride(W, H, S)
    packed = np.full((S * stride * 64, 2), -1, np.int64)
    for k in range(S):
        for t, (tx, ty) in enumerate(multigpu.shard_tiles(W, H, k, S)):
            lane = np.arange(64)
            packed[(k * stride + t) * 64 + lane, 0] = tx * 8 + (lane & 7)
            packed[(k * stride + t) * 64 + lane, 1] = ty * 8 + (lane >> 3)
    frame = multigpu.unpack_tiles_numpy(packed, W, H, S, stride)
    yy, xx = np.mgrid[0:H, 0:W]
    assert np.array_equal(frame[..., 0], xx) and np.array_equal(frame[..., 1], yy)


@pytest.mark.parametrize("W,H,S", [(100, 52, 1), (100, 52, 3), (44, 30, 5), (200, 120, 8), (64, 64, 6)])
def test_shard_tile_index_inverts_the_shard_order(W, H, S):
    """The unpack kernels address the packed buffer from the output tile (shard_tile_index)."""
    for k in range(S):
        for t, (tx, ty) in enumerate(multigpu.shard_tiles(W, H, k, S)):
            assert multigpu.shard_tile_index(int(tx), int(ty), W, H, S) == (k, t)


def test_planar_tiles_restore_the_packed_pixels():
    """BH_LAYOUT_TILES_RGB is BH_LAYOUT_TILES with each tile's pixels split into R, G, B planes and
    alpha dropped; planar_to_packed (the numpy statement of bh_tiles_unpack_rgb's per-tile step)
    inverts it when alpha is the constant."""
    rng = np.random.default_rng(3)
    n = 7
    px = rng.integers(0, 256, (n * 64, 4), dtype=np.uint8)
    px[:, 3] = 255
    planes = px.reshape(n, 64, 4)[..., :3].transpose(0, 2, 1).copy()
    assert planes.shape == (n, 3, 64) and planes.nbytes == px.nbytes * 3 // 4
    assert np.array_equal(multigpu.planar_to_packed(planes, 255), px)
    f = rng.standard_normal((n * 64, 4)).astype(np.float16)
    f[:, 3] = 1.0
    assert np.array_equal(multigpu.planar_to_packed(f.reshape(n, 64, 4)[..., :3].transpose(0, 2, 1), 1.0), f)


def test_weak_scaling_frames():
    assert multigpu.weak_scaling_frame(1) == (4096, 2048)
    assert multigpu.weak_scaling_frame(4) == (8192, 4096)  # BASELINE config 4 frame
    for n in (2, 8):
        w, h = multigpu.weak_scaling_frame(n)
        assert w % 8 == 0 and h % 8 == 0 and abs(w * h / (n * 4096 * 2048) - 1) < 0.01


def test_invalid_arguments_are_status_codes_not_crashes():
    lib = bh.load()
    assert lib.bh_render(None, None, None, None, None) == bh._abi.BH_ERR_INVALID_ARG
    assert lib.bh_create(None, 0, 0, 0, None) == bh._abi.BH_ERR_INVALID_ARG
    assert lib.bh_shard_tile_count(64, 64, 3, 2) == bh._abi.BH_ERR_INVALID_ARG
    assert lib.bh_tiles_unpack(None, None, 0, 0, 0, 0, 16, None) == bh._abi.BH_ERR_INVALID_ARG
    assert lib.bh_uniforms_default(None) == bh._abi.BH_ERR_INVALID_ARG
    assert lib.bh_destroy(None) == 0


def test_create_without_device_fails_loudly():
    """No CPU fallback: with no GPU visible bh_create reports BH_ERR_NO_DEVICE."""
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(bh.BhError) as ei:
        bh.Scene(16, 16, sky=bh.synthetic_sky(64, 32))
    assert ei.value.status == bh._abi.BH_ERR_NO_DEVICE


def test_load_sky_decodes_to_rgba8(tmp_path):
    """load_sky (Texture::from_image, src/texture.rs:11-27): any image file -> (H, W, 4) RGBA8, alpha 255."""
    PIL = pytest.importorskip("PIL.Image")
    sky = bh.synthetic_sky(128, 64)
    PIL.fromarray(sky[..., :3]).save(tmp_path / "sky.png")
    got = bh.load_sky(tmp_path / "sky.png")
    assert got.shape == (64, 128, 4) and np.array_equal(got, sky)
    PIL.fromarray(sky[..., :3]).save(tmp_path / "sky.jpg", quality=95)
    j = bh.load_sky(tmp_path / "sky.jpg")
    assert j.shape == (64, 128, 4) and (j[..., 3] == 255).all()
    assert np.abs(j[..., :3].astype(int) - sky[..., :3]).mean() < 6  # lossy, but the same picture


def test_tile_bytes_of_every_layout():
    """include/bh_render.h: RGBM tiles are the three RGB planes plus one 8-byte blackout mask word."""
    for fmt, bpp in bh.BYTES_PER_PIXEL.items():
        assert bh.tile_bytes(bh.BH_LAYOUT_TILES, fmt) == 64 * bpp
        assert bh.tile_bytes(bh.BH_LAYOUT_TILES_RGB, fmt) == 48 * bpp
        assert bh.tile_bytes(bh.BH_LAYOUT_TILES_RGBM, fmt) == 48 * bpp + 8 == multigpu.rgbm_tile_bytes(fmt)
        assert bh.tile_bytes(bh.BH_LAYOUT_TILES_RGBM, fmt) % 8 == 0  # the mask word stays 8-byte aligned
    with pytest.raises(bh.BhError):
        bh.tile_bytes(bh.BH_LAYOUT_ROWMAJOR, bh.BH_OUT_RGBA16F)
    with pytest.raises(bh.BhError):
        bh.tile_bytes(bh.BH_LAYOUT_TILES_RGBM, 9)


def test_rgbm14_tile_bytes_and_mirror():
    """BH_LAYOUT_TILES_RGBM14: 344 B per RGBA16F tile (86 words, the mask word 8-byte aligned), other
    formats refused; the host mirrors of its store and unpack restore both targets of any RGBA16F frame
    whose channels are in [0, 1] exactly as the RGBM mirrors do."""
    assert bh.tile_bytes(bh.BH_LAYOUT_TILES_RGBM14, bh.BH_OUT_RGBA16F) == 344 == multigpu.RGBM14_TILE_BYTES
    for fmt in (bh.BH_OUT_RGBA32F, bh.BH_OUT_BGRA8_SRGB):
        with pytest.raises(bh.BhError):
            bh.tile_bytes(bh.BH_LAYOUT_TILES_RGBM14, fmt)
    rng = np.random.default_rng(5)
    H, W = 37, 53
    c = rng.random((H, W, 4)).astype(np.float32)
    c[rng.random((H, W)) < 0.1] = 0.0
    c[rng.random((H, W)) < 0.05, :3] = 1.0
    c[0, 0, :3] = [6.1e-5, 5.96e-8, 0.99951]  # smallest normal, smallest subnormal, largest below 1
    c[..., 3] = 1.0
    c16 = c.astype(np.float16)
    zero = ((c[..., 0] * c[..., 0] + c[..., 1] * c[..., 1]) + c[..., 2] * c[..., 2]) < 1.0
    for S, weights in ((1, None), (3, None), (3, [2, 5, 3])):
        stride = multigpu.packed_stride(W, H, S, weights)
        p14 = np.concatenate([multigpu.pack_rgbm14_numpy(c16, zero, k, S, stride, weights) for k in range(S)])
        p16 = np.concatenate([multigpu.pack_rgbm_numpy(c16, zero, k, S, stride, weights) for k in range(S)])
        c1, b1 = multigpu.unpack_rgbm14_numpy(p14, W, H, S, stride, weights)
        c2, b2 = multigpu.unpack_rgbm_numpy(p16, W, H, S, stride, np.float16, 1.0, weights)
        assert np.array_equal(c1.view(np.uint16), c2.view(np.uint16))
        assert np.array_equal(b1.view(np.uint16), b2.view(np.uint16))
    with pytest.raises(ValueError):  # a channel above 1 does not fit 14 bits
        bad = c16.copy()
        bad[1, 1, 0] = 2.0
        multigpu.pack_rgbm14_numpy(bad, zero, 0, 1, multigpu.packed_stride(W, H, 1))


@pytest.mark.parametrize("S", [1, 2, 3, 8])
@pytest.mark.parametrize("dtype,alpha", [(np.float16, 1.0), (np.float32, 1.0), (np.uint8, 255)])
def test_rgbm_pack_unpack_mirror_restores_both_targets(S, dtype, alpha):
    """Host mirrors of the RGBM transport (the march kernel's store, bh_tiles_unpack_rgbm): the gathered
    shards restore col and blackout_col = col with the masked pixels zeroed, alpha restored; partial
    tiles (100 x 52) included.  The mask is what makes blackout exact: it is decided on the fp32 col,
    so a quantised col alone cannot always reproduce it."""
    W, H = 100, 52
    rng = np.random.default_rng(S)
    col = rng.integers(0, 255, (H, W, 4)).astype(dtype) if dtype == np.uint8 else \
        rng.random((H, W, 4)).astype(dtype)
    col[..., 3] = alpha
    zero = rng.random((H, W)) < 0.3
    stride = multigpu.packed_stride(W, H, S)
    packed = np.concatenate([multigpu.pack_rgbm_numpy(col, zero, k, S, stride) for k in range(S)])
    assert packed.shape == (S * stride, multigpu.rgbm_tile_bytes({np.float32: 0, np.float16: 1, np.uint8: 2}[dtype]))
    c, b = multigpu.unpack_rgbm_numpy(packed, W, H, S, stride, dtype, alpha)
    want_b = col.copy()
    want_b[zero, :3] = 0
    assert np.array_equal(c.view(np.uint8), col.view(np.uint8))
    assert np.array_equal(b.view(np.uint8), want_b.view(np.uint8))


def test_scene_wrappers_reject_undersized_buffers():
    """bloom and the unpack wrappers check buffer sizes on the host (a BhError, not an
    out-of-bounds device access); numpy arrays stand in for device tensors (no launch happens)."""
    torch = pytest.importorskip("torch")
    small = torch.zeros(10, dtype=torch.uint8)
    big = torch.zeros(1 << 16, dtype=torch.uint8)
    with pytest.raises(bh.BhError, match="packed"):
        bh.tiles_unpack_rgbm(small, big, None, 16, 16, 2, 4, bh.BH_OUT_BGRA8_SRGB)
    with pytest.raises(bh.BhError, match="out_col"):
        bh.tiles_unpack_rgbm(big, small, None, 16, 16, 2, 4, bh.BH_OUT_BGRA8_SRGB)
    with pytest.raises(bh.BhError, match="out_blackout"):
        bh.tiles_unpack_rgbm(big, big, small, 16, 16, 2, 4, bh.BH_OUT_BGRA8_SRGB)
    with pytest.raises(bh.BhError, match="packed"):
        bh.tiles_unpack_rgb(small, big, 16, 16, 2, 4, bh.BH_OUT_BGRA8_SRGB)
    with pytest.raises(bh.BhError, match="out"):
        bh.tiles_unpack(big, small, 16, 16, 2, 4, 4)
    with pytest.raises(bh.BhError, match="must be contiguous"):
        bh.tiles_unpack(big, big.view(256, 256).t(), 16, 16, 2, 4, 4)
