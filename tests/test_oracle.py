"""CPU tests of the oracle (test infrastructure): golden fixtures, the independent numpy restatement,
and physics known-answer tests.  PARITY UNPINNED against the reference itself (it cannot run here
and ships no fixtures): these pin the restatement by construction and by physics."""
from pathlib import Path

import numpy as np
import pytest

import black_hole_ray_marching_amd as bh
import oracle
from oracle import oracle_np
from tests._cases import camera_uniform, uniforms

GOLDEN = sorted((Path(__file__).parent / "golden").glob("cam*.npz"))


def load_fixture(p):
    z = np.load(p)  # plain arrays only (allow_pickle=False)
    W, H, cap, flags = (int(v) for v in z["meta"])
    return z, W, H, cap, flags


def test_golden_fixtures_present():
    assert len(GOLDEN) >= 8


@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_oracle_matches_golden(path):
    z, W, H, cap, flags = load_fixture(path)
    col, bo, n_rk, fate = oracle.render_rows(z["camera_uniform"].tobytes(), z["uniforms"].tobytes(), z["sky"],
                                             W, H, cap, flags)
    assert np.array_equal(col.view(np.uint32), z["col"].view(np.uint32))
    assert np.array_equal(n_rk, z["n_rk"]) and np.array_equal(fate, z["fate"])
    # blackout target == pure per-pixel function of col (src/black_hole_maybe.wgsl:365-368)
    c = z["col"]
    keep = ~(((c[..., 0] * c[..., 0] + c[..., 1] * c[..., 1]) + c[..., 2] * c[..., 2]) < np.float32(1))
    assert np.array_equal(bo, np.where(keep[..., None], c, np.array([0, 0, 0, 1], np.float32)))


@pytest.mark.parametrize("cam,W,H,cap,flags,over", [
    ("A", 40, 24, 512, 3, {}), ("B", 32, 32, 64, 0, {}), ("C", 40, 20, 1000, 3, {}),
    ("D", 32, 24, 512, 1, {"rs": 1.3}), ("E", 32, 20, 512, 2, {"delta_time_mult": 0.3}),
    ("A", 24, 16, 512, 3, {"blackout_eh": 0, "max_dist": 80.0}),
])
def test_c_oracle_equals_numpy_restatement(sky_small, cam, W, H, cap, flags, over):
    cu, U = camera_uniform(cam, W, H), uniforms(**over)
    col, _, n_rk, fate = oracle.render_rows(cu.to_bytes(), bytes(U.to_c()), sky_small, W, H, cap, flags)
    with np.errstate(all="ignore"):
        c2, _, n2, f2 = oracle_np.render(cu.pos, cu.world_tri, U.as_dict(), sky_small, W, H, cap, flags)
    assert np.array_equal(fate, f2) and np.array_equal(n_rk, n2)
    assert np.array_equal(col.view(np.uint32), c2.view(np.uint32))


def test_row_sampling_matches_full_frame(sky_small):
    cu, U = camera_uniform("B", 64, 40), uniforms()
    full = oracle.render_rows(cu.to_bytes(), bytes(U.to_c()), sky_small, 64, 40, 512, 3)
    band = oracle.render_rows(cu.to_bytes(), bytes(U.to_c()), sky_small, 64, 40, 512, 3, 3, 40, row_step=8)
    assert np.array_equal(band[0], full[0][3::8]) and np.array_equal(band[2], full[2][3::8])


def test_srgb_lut_is_the_standard_decode():
    lut = oracle.srgb_lut()
    c = np.arange(256) / 255.0
    ref = np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4)
    assert np.abs(lut - ref).max() < 1e-7 and lut[0] == 0 and lut[255] == 1


# ---- physics known-answer tests ---------------------------------------------------------------

def _U(**kw):
    u = bh.Uniforms.default()
    for k, v in kw.items():
        setattr(u, k, v)
    return bytes(u.to_c())


def test_kat_shadow_edge_at_critical_impact_parameter(sky_small):
    """Capture iff b < b_c = 3*sqrt(3)/2 * RS (photon sphere at 1.5 RS), RS = 1."""
    bc = 1.5 * np.sqrt(3.0)
    for b in (2.0, 2.4, 2.55, 2.59):
        _, _, fate, _, _ = oracle.trace_ray((b, 0, -100), (0, 0, 1), _U(max_dist=1000.0), sky_small, 1000, 0)
        assert fate == bh.BH_FATE_BLACKOUT, b
    for b in (2.61, 2.7, 3.0, 5.0):
        _, _, fate, _, _ = oracle.trace_ray((b, 0, -100), (0, 0, 1), _U(max_dist=1000.0), sky_small, 1000, 0)
        assert fate == bh.BH_FATE_ESCAPE, b
    assert 2.59 < bc < 2.61


@pytest.mark.parametrize("b", [30.0, 60.0, 120.0])
def test_kat_weak_field_deflection(sky_small, b):
    """Deflection -> 4M/b + 15 pi M^2 / (4 b^2) with M = RS/2 (second-order Schwarzschild)."""
    _, _, fate, ro, rd = oracle.trace_ray((b, 0, -500), (0, 0, 1), _U(max_dist=3000.0), sky_small, 1000, 0)
    assert fate == bh.BH_FATE_ESCAPE
    ang = float(np.arctan2(-rd[0], rd[2]))
    M = 0.5
    expect = 4 * M / b + 15 * np.pi * M * M / (4 * b * b)
    assert abs(ang / expect - 1) < 0.01, (ang, expect)


def test_kat_deflection_scales_with_distortion_power(sky_small):
    base = oracle.trace_ray((40, 0, -500), (0, 0, 1), _U(max_dist=3000.0), sky_small, 1000, 0)[4]
    half = oracle.trace_ray((40, 0, -500), (0, 0, 1), _U(max_dist=3000.0, distortion_power=0.5), sky_small, 1000, 0)[4]
    r = np.arctan2(-half[0], half[2]) / np.arctan2(-base[0], base[2])
    assert abs(r - 0.5) < 0.02


def test_kat_distortion_zero_gives_straight_rays_and_analytic_sky(sky_small):
    """DISTORTION_POWER = 0: rd never changes (bit-for-bit), so escaped pixels sample the sky at
    the initial direction: u = (atan2(z,x)+pi)/2pi, v = 1-(y+1)/2 (src/black_hole_maybe.wgsl:330-343)."""
    W, H = 48, 24
    cu, U = camera_uniform("B", W, H), uniforms(distortion_power=0.0)
    col, _, n_rk, fate = oracle.render_rows(cu.to_bytes(), bytes(U.to_c()), sky_small, W, H, 512, 0)
    rd0 = oracle_np.pixel_dirs(cu.world_tri, W, H)
    with np.errstate(all="ignore"):
        ln = oracle_np._len(rd0[:, 0], rd0[:, 1], rd0[:, 2])
    n = rd0 / ln[:, None]
    u = ((np.arctan2(n[:, 2].astype(np.float64), n[:, 0].astype(np.float64)).astype(np.float32)
          + oracle_np.ONE_PI) / oracle_np.TWO_PI)
    v = np.float32(1) - (n[:, 1] + np.float32(1)) * np.float32(0.5)
    r_, g_, b_ = oracle_np._sample(sky_small, oracle_np.srgb_lut(), u, v)
    exp = np.stack([r_, g_ * np.sqrt(g_), b_ * np.sqrt(b_)], axis=1).reshape(H, W, 3)
    esc = fate == bh.BH_FATE_ESCAPE
    assert esc.mean() > 0.9
    assert np.array_equal(col[..., :3][esc].view(np.uint32), exp[esc].astype(np.float32).view(np.uint32))


def test_kat_straight_ray_hits_marker_sphere(sky_small):
    """DP = 0: a straight ray aimed at the marker centre (10,0,-10) hits its r = 0.5 surface;
    one that passes 1.0 from the centre misses (markers are not scaled by RS: quirk Q5)."""
    d = np.array([10.0, 0.0, 10.0]) / np.sqrt(200.0)
    rgb, _, fate, _, _ = oracle.trace_ray((0, 0, -20), tuple(d), _U(distortion_power=0.0), sky_small, 512, 2)
    assert fate == bh.BH_FATE_SURFACE and np.all(rgb == 1)
    miss = np.array([10.0, 1.0, 10.0]) / np.linalg.norm([10.0, 1.0, 10.0])
    _, _, fate, _, _ = oracle.trace_ray((0, 0, -20), tuple(miss), _U(distortion_power=0.0), sky_small, 512, 2)
    assert fate == bh.BH_FATE_ESCAPE


def test_kat_camera_inside_surface_returns_one_immediately(sky_small):
    """Q9: the first iteration tests surfaces before stepping."""
    cam = bh.Camera.look_at((10.0, 0.0, -10.0), (0.0, 0.0, 0.0), 16, 8)
    cu = bh.CameraUniform()
    cu.update(cam)
    col, _, n_rk, fate = oracle.render_rows(cu.to_bytes(), bytes(uniforms().to_c()), sky_small, 16, 8, 512, 3)
    assert np.all(fate == bh.BH_FATE_SURFACE) and np.all(n_rk == 0) and np.all(col == 1)


def test_kat_cap_still_shades_sky(sky_small):
    W, H = 32, 16
    cu, U = camera_uniform("A", W, H), uniforms()
    col, _, n_rk, fate = oracle.render_rows(cu.to_bytes(), bytes(U.to_c()), sky_small, W, H, 2, 3)
    assert n_rk.max() <= 2 and (fate == bh.BH_FATE_CAP).mean() > 0.9
    capped = fate == bh.BH_FATE_CAP
    assert np.all(col[capped][:, :3] > 0) and np.all(col[..., 3] == 1)


def test_kat_blackout_off_rays_through_origin_are_defined(sky_small):
    """Q8: without blackout a radial ray reaches r = 0 (pow(0, 2.5) = 0 -> inf/NaN); the oracle
    defines a NaN sky coordinate to sample texel (0,0); the result is finite."""
    rgb, n, fate, _, _ = oracle.trace_ray((0, 0, -20), (0, 0, 1), _U(blackout_eh=0), sky_small, 200, 0)
    assert np.all(np.isfinite(rgb))


def test_srgb_encode_table_matches_definition_exhaustively():
    """The BGRA8 output's encoder is the product's 257-entry threshold table (bh_srgb.hpp); the oracle
    checks it against the normative encode (bho_srgb_encode) for every float in [0, 1], and each
    threshold is the exact boundary: code(T[k]) = k and code(prev(T[k])) = k - 1."""
    import black_hole_ray_marching_amd as bh
    T = bh.srgb_encode_table()
    assert T[0] == 0.0 and np.isinf(T[256]) and np.all(np.diff(T) > 0)
    lib = oracle.load()
    for k in range(1, 256):
        prev = np.nextafter(T[k], np.float32(0))
        assert lib.bho_srgb_encode(float(T[k])) == k and lib.bho_srgb_encode(float(prev)) == k - 1, k
    assert oracle.srgb_table_mismatches(T) == 0


def test_srgb_round_trip():
    """A Bgra8UnormSrgb store of a decoded texel gives back its byte: the normative encode of the sRGB
    decode table's entry k is k for every k, and the alpha store unorm8(RN_f32(k / 255)) is k (the
    bloom's literal copy passes store a texel-centre sample as the texel's own word, bh_bloom.hip
    pass_kernel)."""
    lut = oracle.srgb_lut()
    assert np.array_equal(oracle.srgb_encode(lut.astype(np.float32)).astype(np.int64), np.arange(256))
    a = np.arange(256, dtype=np.float32) / np.float32(255.0)  # RN_f32(k / 255): the alpha decode
    assert np.array_equal(np.floor(a.astype(np.float64) * 255.0 + 0.5).astype(np.int64), np.arange(256))


def test_exit_tests_on_r_squared_equal_tests_on_r():
    # The kernel's blackout/outside tests (bh_march.hpp step_bf) read r2 = dot(ro, ro) instead of
    # r = RN(sqrt(r2)) (src/black_hole_maybe.wgsl:271-283 compares r with 1):
    #   r < 1 <=> r2 < 1   and   r > 1 <=> r2 > 1 + 2^-23.
    # RN(sqrt) is monotone, so checking every float in [1/4, 4] (both sides of both thresholds)
    # proves it for all r2; numpy's float32 sqrt is the correctly rounded IEEE sqrt.
    lo, hi = np.float32(0.25).view(np.uint32), np.float32(4.0).view(np.uint32)
    r2 = np.arange(lo, hi + 1, dtype=np.uint32).view(np.float32)
    r = np.sqrt(r2)
    assert r.dtype == np.float32
    assert np.array_equal(r < 1.0, r2 < np.float32(1.0))
    assert np.array_equal(r > 1.0, r2 > np.float32(1.0 + 2.0 ** -23))
    for x in (np.float32(0.0), np.float32(np.inf), np.float32(np.nan)):
        assert (np.sqrt(x) < 1.0) == (x < 1.0) and (np.sqrt(x) > 1.0) == (x > np.float32(1.0 + 2.0 ** -23))


def test_marker_pair_reduction():
    # bh_march.hpp XOps::sdf evaluates the marker term (src/black_hole_maybe.wgsl:107-117) as
    # sqrt(min(qy, qx)) - 0.5 with qy = (x*x + t*t) + zz, t = RN(10 - |y|), qx = (u*u + y*y) + zz,
    # u = RN(10 - |x|): only the sphere on the point's side of each pair can be nearest.  Checked
    # bit for bit against the oracle's four-sphere min on random and adversarial points.
    from oracle import oracle_np as onp
    rng = np.random.default_rng(7)
    f32 = np.float32
    parts = [rng.normal(0, s, (200_000, 3)) for s in (1.0, 10.0, 30.0, 1e3)]
    pts = np.concatenate(parts).astype(f32)
    special = np.array([0.0, -0.0, 10.0, -10.0, 1e-30, -1e-30, 9.999999, -10.000001, 1e19, -1e19,
                        np.inf, -np.inf, np.nan], dtype=f32)
    grid = np.stack(np.meshgrid(special, special, special, indexing="ij"), -1).reshape(-1, 3)
    near = (f32(10.0) + rng.integers(-3, 4, (100_000, 3)).astype(f32) * np.spacing(f32(10.0))).astype(f32)
    near *= rng.choice(np.array([-1, 1], dtype=f32), near.shape)
    pts = np.concatenate([pts, grid, near]).astype(f32)
    px, py, pz = pts[:, 0], pts[:, 1], pts[:, 2]
    with np.errstate(all="ignore"):
        ref = onp._sdf(px, py, pz, f32(1.0), onp.SCENE_MARKERS)
        xx, yy = px * px, py * py
        dz = f32(-10.0) - pz
        zz = dz * dz
        t, u = f32(10.0) - np.abs(py), f32(10.0) - np.abs(px)
        qm = np.fmin((xx + t * t) + zz, (u * u + yy) + zz)
        got = np.sqrt(qm) - f32(0.5)
    assert got.dtype == np.float32 and ref.dtype == np.float32
    both_nan = np.isnan(got) & np.isnan(ref)
    assert np.array_equal(got.view(np.uint32)[~both_nan], ref.view(np.uint32)[~both_nan])
    assert np.array_equal(np.isnan(got), np.isnan(ref))


def test_parity_envelope_variants_leave_the_normative_path_untouched():
    """oracle.render_rows(variant=...) is test infrastructure for DESIGN.md §3's parity envelope: the
    normative path (variant 0, what every parity test uses) is bit-identical through either entry
    point, and the texture-filter variants change colours only, never a ray's fate or step count."""
    import black_hole_ray_marching_amd as bh
    import oracle
    from tests._cases import camera_uniform, uniforms
    sky = bh.synthetic_sky(512, 256)
    W, H = 64, 32
    cu, U = camera_uniform("A", W, H).to_bytes(), bytes(uniforms().to_c())
    ref = oracle.render_rows(cu, U, sky, W, H, 512, 3)
    lib = oracle.load()
    col = np.empty((H, W, 4), np.float32)
    n = np.empty((H, W), np.uint16)
    f = np.empty((H, W), np.uint8)
    import ctypes as C
    assert lib.bho_render_rows_variant(C.create_string_buffer(cu, 112), C.create_string_buffer(U, 32),
                                       np.ascontiguousarray(sky).ctypes.data, 512, 256, W, H, 512, 3, 0, H, 1,
                                       col.ctypes.data, None, n.ctypes.data, f.ctypes.data, 0, 0) == 0
    assert np.array_equal(col.view(np.uint32), ref[0].view(np.uint32))
    for v in (oracle.V_TEX_8BIT, oracle.V_TEX_NEAREST, oracle.V_ATAN2F):
        got = oracle.render_rows(cu, U, sky, W, H, 512, 3, variant=v)
        assert np.array_equal(got[2], ref[2]) and np.array_equal(got[3], ref[3])
        assert not np.array_equal(got[0].view(np.uint32), ref[0].view(np.uint32))
