"""GPU parity: the HIP kernel (through the C ABI) against the CPU oracle on identical inputs.

Bar (DESIGN.md "Parity"):
  * BH_MATH_EXACT: bit-exact — every output word, n_rk and fate identical to oracle/bh_oracle.c.
  * BH_MATH_FAST:  fate and n_rk identical on >= FAST_MATCH_MIN of pixels; on those pixels the
    max |delta| over RGB (fp32 output) < FAST_TOL.  FAST_TOL is NOT the north_star 1e-4: a one-ulp
    change of the final ray direction moves the sky coordinate by ~2e-4 texels, so at single-texel
    stars any non-bit-exact trajectory shows |delta| ~1e-3.  Only BH_MATH_EXACT meets 1e-4 (it is
    bit-exact); BH_MATH_FAST is the documented approximate mode (DESIGN.md "Math modes").
"""
import numpy as np
import pytest

import black_hole_ray_marching_amd as bh
import oracle
from tests._cases import camera_uniform, uniforms

pytestmark = pytest.mark.gpu

FAST_TOL = 5e-3
FAST_MATCH_MIN = 0.999


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def scene_small(torch_cuda, sky_small):
    return bh.Scene(16, 16, sky=sky_small)


def gpu_render(torch, scene, cu, U, W, H, cap, flags, math, fmt=bh.BH_OUT_RGBA32F, blackout=True, schedule=0):
    scene.camera_uniform = cu
    scene.uniforms = U
    scene.max_iters, scene.scene_flags = cap, flags
    ch_dtype = torch.float32 if fmt == bh.BH_OUT_RGBA32F else torch.float16
    col = torch.full((H, W, 4), float("nan"), dtype=ch_dtype, device="cuda")
    bo = torch.full((H, W, 4), float("nan"), dtype=ch_dtype, device="cuda") if blackout else None
    nrk = torch.full((H, W), 0xFFFF, dtype=torch.int32, device="cuda").to(torch.int16)
    fate = torch.full((H, W), 0xFF, dtype=torch.uint8, device="cuda")
    scene.render(col, bo, fmt=fmt, math=math, dbg_n_rk=nrk, dbg_fate=fate, width=W, height=H, schedule=schedule)
    torch.cuda.synchronize()
    return (col.cpu().numpy(), None if bo is None else bo.cpu().numpy(),
            nrk.cpu().numpy().view(np.uint16), fate.cpu().numpy())


def oracle_render(cu, U, sky, W, H, cap, flags, row0=0, row1=None):
    return oracle.render_rows(cu.to_bytes(), bytes(U.to_c()), sky, W, H, cap, flags, row0, row1)


def assert_bitexact(g, o):
    gc, gb, gn, gf = g
    oc, ob, on, of = o
    assert np.array_equal(gf, of), f"fate mismatch at {np.argwhere(gf != of)[:5]}"
    assert np.array_equal(gn, on), f"n_rk mismatch at {np.argwhere(gn != on)[:5]}"
    bad = gc.view(np.uint32) != oc.view(np.uint32)
    assert not bad.any(), f"col mismatch at {np.argwhere(bad)[:5]}: {gc[bad][:4]} vs {oc[bad][:4]}"
    if gb is not None:
        assert np.array_equal(gb.view(np.uint32), ob.view(np.uint32))


def fast_stats(g, o):
    """fate/n_rk match fraction, and max |delta| over matched pixels that did not run to the cap
    (capped rays orbit the photon sphere: chaotic, any rounding difference changes where they end)."""
    gc, _, gn, gf = g
    oc, _, on, of = o
    match = (gf == of) & (gn == on)
    frac = match.mean()
    d = np.abs(gc[..., :3] - oc[..., :3]).max(axis=-1)
    sel = match & (of != bh.BH_FATE_CAP)
    dmax = float(d[sel].max()) if sel.any() else 0.0
    return frac, dmax, match


def on_fate_boundary(fate, mism):
    f = np.pad(fate, 1, mode="edge")
    c = f[1:-1, 1:-1]
    nb = (f[:-2, 1:-1] != c) | (f[2:, 1:-1] != c) | (f[1:-1, :-2] != c) | (f[1:-1, 2:] != c)
    return nb[mism]


CASES = [
    # cam, W, H, cap, flags, uniform overrides
    ("A", 128, 64, 512, 3, {}),
    ("A", 96, 96, 64, 0, {}),                     # BASELINE config 1 shape (no disc), reduced size
    ("B", 120, 68, 256, 3, {}),                   # partial tiles (68 = 8*8 + 4)
    ("C", 128, 64, 1000, 3, {}),
    ("D", 100, 60, 512, 3, {}),
    ("A", 64, 32, 512, 3, {"blackout_eh": 0}),
    ("B", 64, 32, 512, 3, {"distortion_power": 0.0}),
    ("C", 80, 48, 512, 3, {"rs": 1.4, "delta_time_mult": 0.3, "max_dist": 60.0}),
    ("A", 64, 40, 512, 1, {}),                    # disc only
    ("A", 64, 40, 512, 2, {}),                    # markers only
    ("E", 48, 32, 512, 3, {}),                    # shadow-edge zoom: capped "Zeno" rays
    ("E", 64, 40, 1000, 3, {"blackout_eh": 0}),   # ... without blackout (rays reach r ~ 0)
    # the root-free step's gates (bh_host.cpp: skip for dtm > 0 and 0 < rs <= 8; far-field radius from rs
    # and dtm, off for dtm >= 0.62): a far radius near 190, the rs limit, both off
    ("A", 64, 40, 512, 3, {"delta_time_mult": 0.6}),
    ("B", 64, 40, 512, 3, {"rs": 8.0}),
    ("A", 48, 32, 512, 3, {"rs": 9.0, "delta_time_mult": 0.7}),
]


# every schedule, and both builds of the exact kernels (source order / machine-scheduled; the small
# test frames pick the latter by default)
SCHEDULES = [bh.BH_SCHED_PAIR, bh.BH_SCHED_TILE | bh.BH_SCHED_FLAG_ISSUE_ORDER,
             bh.BH_SCHED_TILE | bh.BH_SCHED_FLAG_LATENCY, bh.BH_SCHED_PERSISTENT | bh.BH_SCHED_FLAG_ISSUE_ORDER]


@pytest.mark.parametrize("schedule", SCHEDULES)
@pytest.mark.parametrize("cam,W,H,cap,flags,over", CASES)
def test_exact_bitexact(torch_cuda, scene_small, sky_small, cam, W, H, cap, flags, over, schedule):
    cu, U = camera_uniform(cam, W, H), uniforms(**over)
    g = gpu_render(torch_cuda, scene_small, cu, U, W, H, cap, flags, bh.BH_MATH_EXACT, schedule=schedule)
    o = oracle_render(cu, U, sky_small, W, H, cap, flags)
    assert_bitexact(g, o)


# cameras on both sides of the unit sphere: the general blackout test (r < 1 and ingoing, or !(r > 1)
# after having been outside) and the camera-outside step (SF_CAM_OUT) with rays plunging through r = 1
HORIZON_CASES = [
    ("F", 64, 48, 128, 3, {}),
    ("F", 64, 48, 128, 0, {}),
    ("F", 48, 32, 128, 1, {}),
    ("F2", 64, 48, 128, 3, {}),
    ("G", 64, 48, 128, 3, {}),
    ("G", 64, 48, 128, 0, {}),
    ("H", 64, 48, 128, 3, {}),
    ("H", 64, 48, 128, 0, {}),
    ("H", 64, 48, 128, 3, {"blackout_eh": 0}),
]


@pytest.mark.parametrize("schedule", SCHEDULES)
@pytest.mark.parametrize("cam,W,H,cap,flags,over", HORIZON_CASES)
def test_exact_bitexact_camera_at_horizon(torch_cuda, scene_small, sky_small, cam, W, H, cap, flags, over, schedule):
    cu, U = camera_uniform(cam, W, H), uniforms(**over)
    g = gpu_render(torch_cuda, scene_small, cu, U, W, H, cap, flags, bh.BH_MATH_EXACT, schedule=schedule)
    o = oracle_render(cu, U, sky_small, W, H, cap, flags)
    assert_bitexact(g, o)
    fates = np.bincount(o[3].ravel(), minlength=4)
    assert fates[bh.BH_FATE_ESCAPE] > 0 and (fates[bh.BH_FATE_BLACKOUT] > 0) == (over.get("blackout_eh", 1) != 0)


def _grazing(cam, over):
    """Scenes whose rays mostly graze the photon sphere: camera E zooms on the shadow edge, and a hole of
    rs >= 8 puts the critical impact parameter (3 sqrt(3) / 2 rs = 20.8 at rs = 8) beyond camera B's distance
    (20.2), so the shadow fills the frame."""
    return cam == "E" or over.get("rs", 0.0) >= 8.0


FAST_XFAIL = ("BH_MATH_FAST does not meet SURVEY §8c's fate/n_rk bar on grazing scenes: its v_rsq / v_rcp "
              "cores and FMA contraction differ from the IEEE ops by an ulp, and near the photon sphere the "
              "step map is chaotic, so an ulp becomes a different step count, fate or exit direction (on the box: "
              "10 of 2560 rays at rs = 8, a fate-matched escaped ray's colour by 0.074).  Exact mode, the headline, "
              "is bit-exact there (test_exact_bitexact); DESIGN.md §4")


@pytest.mark.parametrize("cam,W,H,cap,flags,over", [
    pytest.param(*c, marks=pytest.mark.xfail(reason=FAST_XFAIL, strict=False)) if _grazing(c[0], c[5]) else c
    for c in CASES])
def test_fast_tolerance(torch_cuda, scene_small, sky_small, cam, W, H, cap, flags, over):
    """The fast mode's documented bar on every case: fate/n_rk equal on >= FAST_MATCH_MIN of pixels (or at
    most 2 pixels differ), |delta| < FAST_TOL on matched escaped pixels.  The grazing cases are expected to
    miss it (xfail with the recorded cause); test_fast_grazing_envelope bounds how far they miss."""
    cu, U = camera_uniform(cam, W, H), uniforms(**over)
    g = gpu_render(torch_cuda, scene_small, cu, U, W, H, cap, flags, bh.BH_MATH_FAST)
    o = oracle_render(cu, U, sky_small, W, H, cap, flags)
    frac, dmax, match = fast_stats(g, o)
    assert frac >= FAST_MATCH_MIN or (~match).sum() <= 2, f"fate/n_rk match {frac:.5f}"
    assert dmax < FAST_TOL, f"max |delta| on matched escaped pixels {dmax:.3g}"
    # blackout target is the pure per-pixel function of col (:365-368)
    gc, gb = g[0], g[1]
    keep = ~(((gc[..., 0] * gc[..., 0] + gc[..., 1] * gc[..., 1]) + gc[..., 2] * gc[..., 2]) < 1.0)
    exp = np.where(keep[..., None], gc, np.array([0, 0, 0, 1], np.float32))
    assert np.array_equal(gb, exp)


@pytest.mark.parametrize("cam,W,H,cap,flags,over", [c for c in CASES if _grazing(c[0], c[5])])
def test_fast_grazing_envelope(torch_cuda, scene_small, sky_small, cam, W, H, cap, flags, over):
    """How far the fast mode misses on grazing scenes, bounded so that a regression still fails: fate/n_rk
    equal on >= 98 % of pixels, and at most 1 % of the matched escaped pixels above FAST_TOL (ADVICE r4:
    an explicit looser bound instead of none)."""
    cu, U = camera_uniform(cam, W, H), uniforms(**over)
    g = gpu_render(torch_cuda, scene_small, cu, U, W, H, cap, flags, bh.BH_MATH_FAST)
    o = oracle_render(cu, U, sky_small, W, H, cap, flags)
    frac, _, match = fast_stats(g, o)
    assert frac >= 0.98, f"fate/n_rk match {frac:.5f}"
    d = np.abs(g[0][..., :3] - o[0][..., :3]).max(axis=-1)
    sel = match & (o[3] != bh.BH_FATE_CAP)
    over_tol = float((d[sel] >= FAST_TOL).mean()) if sel.any() else 0.0
    assert over_tol <= 0.01, f"{over_tol:.4f} of matched escaped pixels above {FAST_TOL}"


def test_fp16_output_is_rne_of_exact(torch_cuda, scene_small, sky_small):
    W, H, cap = 128, 64, 512
    cu, U = camera_uniform("B", W, H), uniforms()
    g16 = gpu_render(torch_cuda, scene_small, cu, U, W, H, cap, 3, bh.BH_MATH_EXACT, fmt=bh.BH_OUT_RGBA16F)
    oc, ob, _, _ = oracle_render(cu, U, sky_small, W, H, cap, 3)
    assert np.array_equal(g16[0].view(np.uint16), oc.astype(np.float16).view(np.uint16))
    assert np.array_equal(g16[1].view(np.uint16), ob.astype(np.float16).view(np.uint16))


def test_blackout_target_none(torch_cuda, scene_small, sky_small):
    W, H = 64, 32
    cu, U = camera_uniform("A", W, H), uniforms()
    g = gpu_render(torch_cuda, scene_small, cu, U, W, H, 512, 3, bh.BH_MATH_EXACT, blackout=False)
    o = oracle_render(cu, U, sky_small, W, H, 512, 3)
    assert np.array_equal(g[0].view(np.uint32), o[0].view(np.uint32))


@pytest.mark.parametrize("schedule", SCHEDULES)
@pytest.mark.parametrize("S", [1, 2, 3, 5, 8])
def test_tiles_shards_unpack(torch_cuda, scene_small, S, schedule):
    torch = torch_cuda
    W, H = 100, 52
    scene = scene_small
    scene.camera_uniform = camera_uniform("C", W, H)
    scene.uniforms, scene.max_iters, scene.scene_flags = uniforms(), 512, 3
    ref = torch.full((H, W, 4), float("nan"), device="cuda")
    scene.render(ref, None, math=bh.BH_MATH_EXACT, width=W, height=H)
    counts = [bh.shard_tile_count(W, H, k, S) for k in range(S)]
    tiles_x, tiles_y = (W + 7) // 8, (H + 7) // 8
    assert sum(counts) == tiles_x * tiles_y
    stride = max(counts)
    packed = torch.full((S * stride * 64, 4), float("nan"), device="cuda")
    for k in range(S):
        part = packed[k * stride * 64:(k + 1) * stride * 64]
        scene.render(part, None, math=bh.BH_MATH_EXACT, layout=bh.BH_LAYOUT_TILES, shard_index=k,
                     shard_count=S, width=W, height=H, schedule=schedule)
    out = torch.full((H, W, 4), float("nan"), device="cuda")
    bh.tiles_unpack(packed, out, W, H, S, stride, 16)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))


@pytest.mark.parametrize("fmt", [bh.BH_OUT_RGBA32F, bh.BH_OUT_RGBA16F, bh.BH_OUT_BGRA8_SRGB])
@pytest.mark.parametrize("S", [1, 3, 8])
def test_tiles_rgb_shards_unpack(torch_cuda, scene_small, S, fmt):
    """BH_LAYOUT_TILES_RGB (the multi-GPU transport, alpha dropped): each shard's planes equal the
    BH_LAYOUT_TILES pixels less alpha, for col and blackout, and bh_tiles_unpack_rgb of the gathered
    shards reproduces the row-major frame word for word (alpha restored)."""
    from black_hole_ray_marching_amd.multigpu import planar_to_packed
    torch = torch_cuda
    W, H = 100, 52
    dt = {bh.BH_OUT_RGBA32F: torch.float32, bh.BH_OUT_RGBA16F: torch.float16, bh.BH_OUT_BGRA8_SRGB: torch.uint8}[fmt]
    alpha = 255 if fmt == bh.BH_OUT_BGRA8_SRGB else 1.0
    scene = scene_small
    scene.camera_uniform = camera_uniform("C", W, H)
    scene.uniforms, scene.max_iters, scene.scene_flags = uniforms(), 512, 3
    ref = torch.zeros((H, W, 4), dtype=dt, device="cuda")
    scene.render(ref, None, fmt=fmt, width=W, height=H)
    stride = max(bh.shard_tile_count(W, H, k, S) for k in range(S))
    planes = torch.zeros((S * stride, 3, 64), dtype=dt, device="cuda")
    for k in range(S):
        n = bh.shard_tile_count(W, H, k, S)
        px_c = torch.zeros((n * 64, 4), dtype=dt, device="cuda")
        px_b = torch.zeros_like(px_c)
        pl_b = torch.zeros((n, 3, 64), dtype=dt, device="cuda")
        kw = dict(fmt=fmt, shard_index=k, shard_count=S, width=W, height=H)
        scene.render(planes[k * stride:k * stride + n], pl_b, layout=bh.BH_LAYOUT_TILES_RGB, **kw)
        scene.render(px_c, px_b, layout=bh.BH_LAYOUT_TILES, **kw)
        torch.cuda.synchronize()
        for pl, px in ((planes[k * stride:k * stride + n], px_c), (pl_b, px_b)):
            # pixels outside the frame are untouched in both layouts (zeros), alpha included
            got = planar_to_packed(pl.cpu().numpy(), alpha)
            want = px.cpu().numpy().copy()
            want[..., 3] = alpha
            assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    # all tile rows at once, and throttled to 2 rows in flight (bh_tiles_unpack_rgb_rows: the
    # kernel grid-strides over the 7 tile rows)
    for rows in (0, 2):
        out = torch.zeros((H, W, 4), dtype=dt, device="cuda")
        bh.tiles_unpack_rgb(planes, out, W, H, S, stride, fmt, rows_in_flight=rows)
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.uint8), ref.view(torch.uint8)), f"rows_in_flight={rows}"


def test_headline_rows_bitexact_and_fast(torch_cuda):
    """4096x2048, cap 512, camera A, full sky: sampled rows through the full-size launch."""
    torch = torch_cuda
    W, H, cap = 4096, 2048, 512
    sky = bh.synthetic_sky()
    scene = bh.Scene(W, H, sky=sky, max_iters=cap)
    cu = scene.camera_uniform
    rows = [0, 517, 1023, 1024, 1100, 2047]
    for math in (bh.BH_MATH_EXACT, bh.BH_MATH_FAST):
        col = torch.empty((H, W, 4), device="cuda")
        bo = torch.empty((H, W, 4), device="cuda")
        nrk = torch.empty((H, W), dtype=torch.int16, device="cuda")
        fate = torch.empty((H, W), dtype=torch.uint8, device="cuda")
        scene.render(col, bo, math=math, dbg_n_rk=nrk, dbg_fate=fate)
        torch.cuda.synchronize()
        for r in rows:
            o = oracle_render(cu, scene.uniforms, sky, W, H, cap, 3, r, r + 1)
            g = (col[r:r + 1].cpu().numpy(), bo[r:r + 1].cpu().numpy(),
                 nrk[r:r + 1].cpu().numpy().view(np.uint16), fate[r:r + 1].cpu().numpy())
            if math == bh.BH_MATH_EXACT:
                assert_bitexact(g, o)
            else:
                frac, dmax, _ = fast_stats(g, o)
                assert frac >= 0.998 and dmax < FAST_TOL, (r, frac, dmax)
        # size-independent property: every pixel got a valid fate, n_rk <= cap, alpha == 1
        f = fate.cpu().numpy()
        assert f.max() <= 3
        assert int(nrk.cpu().numpy().view(np.uint16).max()) <= cap
        assert bool((col[..., 3] == 1).all())
    scene.close()


def test_invalid_arguments_fail_loudly(torch_cuda, scene_small):
    torch = torch_cuda
    out = torch.empty((8, 8, 4), device="cuda")
    with pytest.raises(bh.BhError):
        scene_small.render(out, None, width=8, height=8, shard_count=2)  # row-major needs 1 shard
    with pytest.raises(bh.BhError):
        scene_small.render(out, None, width=8, height=8, fmt=7)
    cu = bh.CameraUniform()
    cu.c.screen_tri[0][0] = 2.0
    old = scene_small.camera_uniform
    scene_small.camera_uniform = cu
    with pytest.raises(bh.BhError):
        scene_small.render(out, None, width=8, height=8)
    scene_small.camera_uniform = old


GOLDEN = sorted((__import__("pathlib").Path(__file__).parent / "golden").glob("cam*.npz"))


@pytest.mark.parametrize("schedule", SCHEDULES)
@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_exact_matches_golden_fixtures(torch_cuda, path, schedule):
    torch = torch_cuda
    z = np.load(path)
    W, H, cap, flags = (int(v) for v in z["meta"])
    scene = bh.Scene(W, H, sky=z["sky"], max_iters=cap, scene_flags=flags, math=bh.BH_MATH_EXACT)
    cu = bh.CameraUniform()
    C = __import__("ctypes")
    C.memmove(C.addressof(cu.c), z["camera_uniform"].tobytes(), 112)
    scene.camera_uniform = cu
    u = bh._abi.bh_uniforms.from_buffer_copy(z["uniforms"].tobytes())
    scene.uniforms = bh.Uniforms(u.rs, u.delta_time_mult, u.bg_brightness, u.blackout_eh, u.max_dist,
                                 u.distortion_power)
    col = torch.full((H, W, 4), float("nan"), device="cuda")
    nrk = torch.zeros((H, W), dtype=torch.int16, device="cuda")
    fate = torch.full((H, W), 0xFF, dtype=torch.uint8, device="cuda")
    scene.render(col, None, dbg_n_rk=nrk, dbg_fate=fate, schedule=schedule)
    torch.cuda.synchronize()
    assert np.array_equal(fate.cpu().numpy(), z["fate"])
    assert np.array_equal(nrk.cpu().numpy().view(np.uint16), z["n_rk"])
    assert np.array_equal(col.cpu().numpy().view(np.uint32), z["col"].view(np.uint32))
    scene.close()


def test_temporal_order_never_changes_results(torch_cuda, sky_small):
    """The tile schedule orders dispatch by the previous frame's per-tile cost.  Costs learned on
    one camera and reused on another, and the static centre-out order, give identical bits."""
    torch = torch_cuda
    W, H, cap = 160, 96, 512
    scene = bh.Scene(W, H, sky=sky_small, max_iters=cap, math=bh.BH_MATH_EXACT)
    outs = {}
    for name, cam, sched in [("E1", "E", bh.BH_SCHED_TILE), ("A_after_E", "A", bh.BH_SCHED_TILE),
                             ("A_again", "A", bh.BH_SCHED_TILE),
                             ("A_static", "A", bh.BH_SCHED_TILE | bh.BH_SCHED_FLAG_STATIC_ORDER)]:
        scene.camera_uniform = camera_uniform(cam, W, H)
        col = torch.full((H, W, 4), float("nan"), device="cuda")
        nrk = torch.zeros((H, W), dtype=torch.int16, device="cuda")
        scene.render(col, None, dbg_n_rk=nrk, schedule=sched)
        torch.cuda.synchronize()
        outs[name] = (col.cpu().numpy(), nrk.cpu().numpy())
    for k in ("A_again", "A_static"):
        assert np.array_equal(outs[k][0].view(np.uint32), outs["A_after_E"][0].view(np.uint32))
        assert np.array_equal(outs[k][1], outs["A_after_E"][1])
    o = oracle_render(camera_uniform("A", W, H), uniforms(), sky_small, W, H, cap, 3)
    assert np.array_equal(outs["A_after_E"][0].view(np.uint32), o[0].view(np.uint32))
    scene.close()


@pytest.mark.parametrize("W,H", [(1024, 1024), (1496, 1000)])
def test_temporal_order_is_a_permutation_across_blocks(torch_cuda, sky_small, W, H):
    """The order kernel sorts ORDER_PER_BLOCK (4096) slots per block and reserves bucket ranges
    with global atomics: at several blocks (and a partial last block), frames rendered in the
    learned order cover every tile exactly once (NaN-filled targets) and equal the static order."""
    torch = torch_cuda
    cap = 64
    scene = bh.Scene(W, H, sky=sky_small, max_iters=cap, math=bh.BH_MATH_EXACT)
    ref = None
    for i, cam in enumerate(["B", "A", "A", "E", "A"]):
        scene.camera_uniform = camera_uniform(cam, W, H)
        col = torch.full((H, W, 4), float("nan"), device="cuda")
        scene.render(col, None, schedule=bh.BH_SCHED_TILE)
        torch.cuda.synchronize()
        if cam != "A":
            continue
        got = col.cpu().numpy().view(np.uint32)
        if ref is None:
            st = torch.full((H, W, 4), float("nan"), device="cuda")
            scene.render(st, None, schedule=bh.BH_SCHED_TILE | bh.BH_SCHED_FLAG_STATIC_ORDER)
            torch.cuda.synchronize()
            ref = st.cpu().numpy().view(np.uint32)
            assert not np.isnan(st.cpu().numpy()).any()
        assert np.array_equal(got, ref), f"frame {i}"
    scene.close()


def test_repeated_frames_skip_the_order_build_and_stay_exact(torch_cuda, sky_small):
    """A launch whose frame repeats the one the dispatch order was learned from runs no order build and
    writes no costs (bh_host.cpp, OrderState::order_key); every path keeps the counters holding the
    histogram of the stored costs, also in graphs captured either way (a march alone, or build + writing
    march) and replayed between eager renders of other cameras.  Every frame covers every tile once
    (NaN-filled targets, a partial last order block) and equals the static order's bytes."""
    torch = torch_cuda
    W, H, cap = 1496, 1000, 64
    scene = bh.Scene(W, H, sky=sky_small, max_iters=cap, math=bh.BH_MATH_EXACT)
    s = torch.cuda.Stream()
    refs = {}
    for cam in ("A", "B", "E"):
        scene.camera_uniform = camera_uniform(cam, W, H)
        st = torch.full((H, W, 4), float("nan"), device="cuda")
        scene.render(st, None, schedule=bh.BH_SCHED_TILE | bh.BH_SCHED_FLAG_STATIC_ORDER, stream=s)
        torch.cuda.synchronize()
        assert not torch.isnan(st).any()
        refs[cam] = st.view(torch.int32).clone()
    out = torch.empty((H, W, 4), device="cuda")

    def eager(cam, i):
        scene.camera_uniform = camera_uniform(cam, W, H)
        out.fill_(float("nan"))
        scene.render(out, None, stream=s)
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int32), refs[cam]), f"eager {cam} #{i}"

    def captured(cam, replays):
        scene.camera_uniform = camera_uniform(cam, W, H)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            scene.render(out, None, stream=s)
        for r in range(replays):
            out.fill_(float("nan"))
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(out.view(torch.int32), refs[cam]), f"replay {cam} #{r}"
        return g

    for i in range(3):
        eager("A", i)            # build + write twice (fresh costs, then A's), then a repeat: neither
    gA = captured("A", 3)        # a repeat captured: a march that writes nothing
    eager("B", 0)                # build (from A's costs) + write B's
    gB = captured("B", 3)        # build (from B's costs) + writing march, per replay
    for i, cam in enumerate(["A", "A", "E", "B", "B", "B", "A"]):
        eager(cam, i)
    for g, cam in ((gA, "A"), (gB, "B")):
        scene.camera_uniform = camera_uniform(cam, W, H)
        out.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int32), refs[cam]), f"late replay {cam}"
    eager("E", 9)
    scene.close()


@pytest.mark.parametrize("cam", ["A", "B"])
def test_cycle_fast_forward_is_exact(torch_cuda, cam):
    """The tile schedule advances rays caught in an exact period-1/2 cycle straight to the cap
    (DESIGN.md "Cycle fast-forward").  At the headline size: some rays are fast-forwarded
    (dbg_steps < dbg_n_rk), only capped ones, and the frame is bit-identical to the pair schedule
    (which iterates every step) and, on every row holding a fast-forwarded ray, to the oracle."""
    torch = torch_cuda
    W, H, cap = 4096, 2048, 512
    sky = bh.synthetic_sky()
    scene = bh.Scene(W, H, sky=sky, max_iters=cap, math=bh.BH_MATH_EXACT)
    scene.camera_uniform = camera_uniform(cam, W, H)
    outs = {}
    for sched in (bh.BH_SCHED_TILE, bh.BH_SCHED_PAIR):
        col = torch.full((H, W, 4), float("nan"), device="cuda")
        bo = torch.full((H, W, 4), float("nan"), device="cuda")
        nrk = torch.zeros((H, W), dtype=torch.int16, device="cuda")
        steps = torch.zeros((H, W), dtype=torch.int16, device="cuda")
        fate = torch.full((H, W), 0xFF, dtype=torch.uint8, device="cuda")
        scene.render(col, bo, dbg_n_rk=nrk, dbg_fate=fate, dbg_steps=steps, schedule=sched)
        torch.cuda.synchronize()
        outs[sched] = (col.cpu().numpy(), bo.cpu().numpy(), nrk.cpu().numpy().view(np.uint16),
                       fate.cpu().numpy(), steps.cpu().numpy().view(np.uint16))
    t, p = outs[bh.BH_SCHED_TILE], outs[bh.BH_SCHED_PAIR]
    for k in range(4):
        assert np.array_equal(t[k].view(np.uint8), p[k].view(np.uint8)), k
    nrk, fate, steps = t[2], t[3], t[4]
    ff = steps != nrk
    assert np.array_equal(p[4], p[2])            # pair: no fast-forward
    assert ff.sum() > 100, ff.sum()              # cameras A/B: ~800 / ~1100 cycling rays
    assert (steps <= nrk).all() and (fate[ff] == bh.BH_FATE_CAP).all() and (nrk[ff] == cap).all()
    rows = np.unique(np.nonzero(ff)[0])
    for r0 in rows[:: max(1, len(rows) // 12)]:
        o = oracle_render(camera_uniform(cam, W, H), uniforms(), sky, W, H, cap, 3, int(r0), int(r0) + 1)
        assert_bitexact(tuple(x[r0:r0 + 1] for x in t[:4]), o)
    scene.close()


def _bgra8_expected(col_f32):
    enc = oracle.srgb_encode(col_f32[..., :3])
    out = np.empty(col_f32.shape[:-1] + (4,), np.uint8)
    out[..., 0], out[..., 1], out[..., 2], out[..., 3] = enc[..., 2], enc[..., 1], enc[..., 0], 255
    return out


@pytest.mark.parametrize("schedule", SCHEDULES)
@pytest.mark.parametrize("cam", ["A", "D"])
def test_bgra8_srgb_output_is_encoded_exact_result(torch_cuda, sky_small, cam, schedule):
    """BH_OUT_BGRA8_SRGB (the reference's Bgra8UnormSrgb targets): every byte equals the normative
    encode (oracle bho_srgb_encode) of the oracle's fp32 colour, for col and blackout_col."""
    torch = torch_cuda
    W, H, cap = 136, 72, 512
    scene = bh.Scene(W, H, sky=sky_small, max_iters=cap, math=bh.BH_MATH_EXACT)
    scene.camera_uniform = camera_uniform(cam, W, H)
    col = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    bo = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    scene.render(col, bo, fmt=bh.BH_OUT_BGRA8_SRGB, schedule=schedule)
    torch.cuda.synchronize()
    o = oracle_render(camera_uniform(cam, W, H), uniforms(), sky_small, W, H, cap, 3)
    assert np.array_equal(col.cpu().numpy(), _bgra8_expected(o[0]))
    assert np.array_equal(bo.cpu().numpy(), _bgra8_expected(o[1]))
    scene.close()


@pytest.mark.parametrize("env", [{"BH_NO_SDF_SKIP": "1"}, {"BH_ORDER_ALWAYS": "1"}], ids=["no_sdf_skip", "order_always"])
def test_march_switches_stay_bitexact(torch_cuda, env):
    """The march's two run-time A/B switches, which the library reads once per process, in a child process each:
    every step evaluates its SDF roots (no root-free step), and the temporal order rebuilt on every launch (no
    repeat skip) -- cameras A and E, three frames each, against the oracle bit for bit (tests/_march_env_check.py)."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    e = dict(os.environ, **env)
    e["PYTHONPATH"] = str(root) + os.pathsep + e.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-m", "tests._march_env_check"], cwd=str(root), env=e, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
