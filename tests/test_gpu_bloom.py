"""GPU parity of the post-processing chain (bh_bloom: Kawase bloom + remix)
against oracle/bh_bloom_oracle.c: bit-exact BGRA8 bytes, fused and literal schedules."""
import numpy as np
import pytest

import black_hole_ray_marching_amd as bh
import oracle
from tests._cases import camera_uniform, uniforms

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _img(rng, H, W, sparse=False):
    t = rng.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
    if sparse:
        t[..., :3] = np.where(rng.random((H, W, 1)) < 0.05, t[..., :3], 0)
    t[..., 3] = 255
    return t


def _gpu_bloom(torch, scene, col, bo, levels, schedule):
    H, W = col.shape[:2]
    c, b = torch.from_numpy(col).cuda(), torch.from_numpy(bo).cuda()
    out = torch.zeros_like(c)
    scene.bloom(c, b, out, levels=levels, schedule=schedule, width=W, height=H)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("schedule", [bh.BH_BLOOM_AUTO, bh.BH_BLOOM_LITERAL])
@pytest.mark.parametrize("H,W,levels", [(128, 256, 3), (64, 64, 1), (64, 128, 2), (120, 200, 3), (37, 53, 3),
                                        (256, 512, 5), (512, 1024, 4), (2048, 4096, 3),
                                        # 2:1 up form (Up2Plan) on thin / narrow power-of-two frames: the
                                        # general sampler's outer ring covers whole axes at the small levels
                                        (32, 2048, 3), (1024, 64, 4), (8, 1024, 2), (64, 16, 3),
                                        # odd widths whose same-size sampling is exact (fused chain): the
                                        # quad kernels' paired stores must not assume 8-byte aligned rows
                                        (64, 65, 3), (33, 129, 3), (65, 33, 2),
                                        # display sizes (config 2's frame; the reference's 1280x720 window,
                                        # src/lib.rs:60-61): same-size passes proven identities, so AUTO
                                        # fuses them; the up passes take the separable plan (per-column /
                                        # per-row taps from the host); also thin frames
                                        (1080, 1920, 3), (720, 1280, 3), (1080, 1920, 5), (7, 300, 3), (300, 7, 3),
                                        # the Y epilogue's in-block fix with a residual fix-up list (1366: at
                                        # every grid origin some inexact columns cross a block edge; 3 at the
                                        # best) and nonzero grid origins (1920: 8, 720 rows: 14)
                                        (768, 1366, 3),
                                        # common display widths the CPU sweep (1..2100) does not reach:
                                        # their strip tables and records
                                        (1440, 2560, 3), (2160, 3840, 3),
                                        # sizes whose same-size copies are not identities (3840x2160, 3440x1440,
                                        # 3840x1080, 1000x700): the general chain with the copies as passes
                                        (1440, 3440, 3), (1080, 3840, 3), (2160, 3840, 1), (2160, 3840, 4), (700, 1000, 2),
                                        (661, 2795, 1), (890, 2057, 2), (615, 2685, 3), (1017, 3121, 4),
                                        # round 6's random-size sweep: the fix-up's dead lanes read far past
                                        # the texture at 3996x495 (a memory fault), harmlessly at 1868x83
                                        # (DESIGN.md §7b); wrong bytes of the removed Y in-block fix at 1846x1392
                                        (495, 3996, 1), (83, 1868, 1), (1392, 1846, 3), (656, 1261, 5),
                                        # the 65536 side limit (a refused plan must fall back to
                                        # the general kernel, not fail the call; tests/test_bloom_bounds.py)
                                        (8, 65536, 3), (65536, 8, 3), (6, 65535, 2)])
def test_bloom_bitexact(torch_cuda, sky_small, H, W, levels, schedule):
    """AUTO fuses the chain: its same-size copies vanish where they are provably identities on stored texels
    (the host's same_size_identity; powers of two trivially) and run as the reference's copy passes where not
    (3840x2160, 3440x1440, ...); LITERAL always runs the pass list.  Both must give the oracle's bytes.  Power-of-two
    sizes also take the 8-tap passes' TapPlan form (constant-offset taps) and the 2:1 up passes'
    Up2Plan form (per-parity offsets and weights), up to the full 4096x2048 frame."""
    rng = np.random.default_rng(W * 7 + H + levels)
    col, bo = _img(rng, H, W), _img(rng, H, W, sparse=True)
    scene = bh.Scene(16, 16, sky=sky_small)
    got = _gpu_bloom(torch_cuda, scene, col, bo, levels, schedule)
    want = oracle.bloom(col, bo, levels)
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    scene.close()


@pytest.mark.parametrize("H,W,levels,sparse", [(128, 256, 3, False), (256, 512, 3, False), (120, 200, 3, False),
                                               (256, 512, 3, True), (512, 1024, 3, True),
                                               # the general fused chain's quad passes and in-block fix
                                               # with alpha below 255 (no opaque-block form)
                                               (1080, 1920, 3, False), (720, 1280, 3, True), (768, 1366, 3, False)])
def test_bloom_bitexact_any_alpha(torch_cuda, sky_small, H, W, levels, sparse):
    """Inputs with every alpha byte (the march writes 255, but bh_bloom takes any BGRA8 texels): the
    exact fma forms of the standard-plan kernels (acc_scaled, clerp, remix) rest on the products by
    powers of two being exact for every decoded channel, alpha k/255 included.  `sparse`: alpha 255
    except at a few scattered texels, so that the final pass runs its opaque-block form (alpha folded)
    and its general form side by side in one frame."""
    rng = np.random.default_rng(W * 3 + H + int(sparse))
    col, bo = _img(rng, H, W), _img(rng, H, W, sparse=True)
    for t in (col, bo):
        a = rng.integers(0, 256, size=(H, W), dtype=np.uint8)
        t[..., 3] = np.where(rng.random((H, W)) < 0.0005, a, 255) if sparse else a
    scene = bh.Scene(16, 16, sky=sky_small)
    for schedule in (bh.BH_BLOOM_AUTO, bh.BH_BLOOM_LITERAL):
        got = _gpu_bloom(torch_cuda, scene, col, bo, levels, schedule)
        want = oracle.bloom(col, bo, levels)
        assert np.array_equal(got, want), (schedule, np.argwhere(got != want)[:5])
    scene.close()


def test_render_then_bloom_matches_oracle_chain(torch_cuda, sky_small):
    """The reference's frame: Scene::render into the two Bgra8UnormSrgb targets, then
    Bloom::render to the surface -- GPU end to end vs the two oracles end to end."""
    torch = torch_cuda
    W, H, cap = 512, 256, 512
    scene = bh.Scene(W, H, sky=sky_small, max_iters=cap, math=bh.BH_MATH_EXACT)
    col = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    bo = torch.zeros_like(col)
    out = torch.zeros_like(col)
    scene.render(col, bo, fmt=bh.BH_OUT_BGRA8_SRGB)
    scene.bloom(col, bo, out)
    torch.cuda.synchronize()
    o = oracle.render_rows(camera_uniform("A", W, H).to_bytes(), bytes(uniforms().to_c()), sky_small, W, H, cap, 3)

    def bgra(c):
        e = oracle.srgb_encode(c[..., :3])
        return np.stack([e[..., 2], e[..., 1], e[..., 0], np.full(e.shape[:2], 255, np.uint8)], -1)
    oc, ob = bgra(o[0]), bgra(o[1])
    assert np.array_equal(col.cpu().numpy(), oc) and np.array_equal(bo.cpu().numpy(), ob)
    assert np.array_equal(out.cpu().numpy(), oracle.bloom(oc, ob, 3))
    scene.close()


def test_no_plan_was_refused(torch_cuda, sky_small):
    """Every plan a real bh_bloom builds is checked on the host before upload (records, strips); a refused plan
    would run the general kernel -- the same bytes, slower -- so the tests' display sizes must refuse none
    (bh_bloom_plan_failures counts them process-wide)."""
    torch = torch_cuda
    scene = bh.Scene(16, 16, sky=sky_small)
    for H, W in ((1080, 1920), (720, 1280), (1440, 2560), (2160, 3840), (768, 1366), (2048, 4096)):
        t = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        scene.bloom(t, t, torch.empty_like(t), width=W, height=H)
    torch.cuda.synchronize()
    n, last = bh.bloom_plan_failures()
    assert n == 0, last
    scene.close()


def test_bloom_invalid_arguments(torch_cuda, sky_small):
    scene = bh.Scene(16, 16, sky=sky_small)
    t = torch_cuda.zeros((16, 16, 4), dtype=torch_cuda.uint8, device="cuda")
    with pytest.raises(bh.BhError):
        scene.bloom(t, t, t, levels=0)
    with pytest.raises(bh.BhError):
        scene.bloom(t, t, t, schedule=7)
    big = torch_cuda.zeros((1, 65537, 4), dtype=torch_cuda.uint8, device="cuda")
    with pytest.raises(bh.BhError):  # width, height <= 65536: the kernels index texels with 32 bits
        scene.bloom(big, big, big, width=65537, height=1)
    scene.close()


# seeded random frame sizes (both sides 1..3300, levels 1..5): whatever fused form, plan, fix-up list and copy
# pass the host picks for them, AUTO must give the oracle's bytes
_RNG_SIZES = np.random.default_rng(20261018)
RANDOM_SIZES = [(int(_RNG_SIZES.integers(1, 1300)), int(_RNG_SIZES.integers(1, 3300)), int(_RNG_SIZES.integers(1, 6)))
                for _ in range(16)]


@pytest.mark.parametrize("H,W,levels", RANDOM_SIZES, ids=[f"{h}x{w}L{l}" for h, w, l in RANDOM_SIZES])
def test_bloom_bitexact_random_sizes(torch_cuda, sky_small, H, W, levels):
    rng = np.random.default_rng(W * 31 + H * 7 + levels)
    col, bo = _img(rng, H, W), _img(rng, H, W, sparse=True)
    scene = bh.Scene(16, 16, sky=sky_small)
    got = _gpu_bloom(torch_cuda, scene, col, bo, levels, bh.BH_BLOOM_AUTO)
    want = oracle.bloom(col, bo, levels)
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    scene.close()


BLOOM_GOLDEN = sorted((__import__("pathlib").Path(__file__).parent / "golden").glob("bloom_*.npz"))


GENERAL_FRAMES = ["1080x1920", "1080x1920:any", "720x1280:any", "768x1366", "768x1366:any"]
STANDARD_FRAMES = ["512x1024", "256x512:any", "2048x4096"]  # powers of two: the standard plans' kernels


@pytest.mark.parametrize("env,frames", [
    ({"BH_BLOOM_FIX2": "1"}, GENERAL_FRAMES),
    ({"BH_BLOOM_ORG_KEEP": "1"}, GENERAL_FRAMES), ({"BH_BLOOM_NO_STRIPS": "1"}, GENERAL_FRAMES),
    ({"BH_BLOOM_FIXUP_NOREC": "1"}, GENERAL_FRAMES), ({"BH_BLOOM_FIXUP_SAMPLE": "1"}, GENERAL_FRAMES),
    ({"BH_BLOOM_NO_SEPQ": "1"}, GENERAL_FRAMES), ({"BH_BLOOM_NO_SEP": "1"}, GENERAL_FRAMES),
    ({"BH_BLOOM_SEPQ_RAW": "3"}, GENERAL_FRAMES), ({"BH_BLOOM_SEPQ_MIN_BLOCKS": "100000"}, GENERAL_FRAMES),
    ({"BH_BLOOM_CAP_PLAIN": "2", "BH_BLOOM_CAP_Y": "2", "BH_BLOOM_CAP_FINAL": "2"}, GENERAL_FRAMES),
    ({"BH_BLOOM_NO_STD": "1"}, STANDARD_FRAMES), ({"BH_BLOOM_NO_UP2": "1"}, STANDARD_FRAMES),
    ({"BH_BLOOM_NO_YQUAD": "1"}, STANDARD_FRAMES), ({"BH_BLOOM_NO_DOWN2": "1"}, STANDARD_FRAMES),
    ({"BH_BLOOM_PERSIST": "1"}, STANDARD_FRAMES), ({"BH_BLOOM_NO_YDOWN2": "1"}, STANDARD_FRAMES),
    ({"BH_BLOOM_NO_GENERAL_COPIES": "1"}, ["1080x3840", "700x1000:any"])],
    ids=["fix2", "org_keep", "no_strips", "fixup_norec", "fixup_sample", "no_sepq", "no_sep", "sepq_raw",
         "sepq_min_blocks", "cap", "no_std", "no_up2", "no_yquad", "no_down2", "persist",
         "no_ydown2", "no_general_copies"])
def test_bloom_switches_stay_bitexact(torch_cuda, env, frames):
    """Every run-time A/B switch of the chain (the library reads them once per process), in a child process each,
    against the oracle bit for bit: on display sizes (the general fused chain: the final epilogue's in-block fix,
    grid origins that keep the block count, the final fix-up from the row-major textures instead
    of its column strips, the fix-up without its records, its per-sample form, the one-pixel separable kernel,
    the per-pixel sampler, raw tiles, quad passes capped in blocks per CU) and on powers of two (the standard
    plans: off, the general up pass instead of the 2:1 form, the Y pass one pixel per lane, no fused double
    downsample, the persistent blocks, the two downsamples in their own pass instead of the Y pass), and sizes whose
    same-size copies are not identities through the literal pass list instead of the general chain."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    e = dict(os.environ, **env)
    e["PYTHONPATH"] = str(root) + os.pathsep + e.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, str(root / "tests" / "_bloom_env_check.py"), *frames], env=e,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("schedule", [bh.BH_BLOOM_AUTO, bh.BH_BLOOM_LITERAL])
@pytest.mark.parametrize("path", BLOOM_GOLDEN, ids=[p.stem for p in BLOOM_GOLDEN])
def test_bloom_matches_golden(torch_cuda, sky_small, path, schedule):
    z = np.load(path)
    scene = bh.Scene(16, 16, sky=sky_small)
    got = _gpu_bloom(torch_cuda, scene, z["col"], z["blackout"], int(z["levels"][0]), schedule)
    assert np.array_equal(got, z["out"])
    scene.close()


def test_bloom_graph_contract(torch_cuda, sky_small):
    """Graph contract of bh_bloom (include/bh_render.h): the first call of a (size, levels, schedule)
    allocates and is refused on a capturing stream; a captured chain's scratch set survives any number of
    other sizes (beyond BH_BLOOM_SETS) and its replay writes the same bytes as a direct call."""
    torch = torch_cuda
    rng = np.random.default_rng(11)
    H, W = 72, 136  # not a power of two: the fused chain's up passes run from separable plans
    col, bo = _img(rng, H, W), _img(rng, H, W, sparse=True)
    c, b = torch.from_numpy(col).cuda(), torch.from_numpy(bo).cuda()
    out = torch.zeros_like(c)
    scene = bh.Scene(16, 16, sky=sky_small)
    s = torch.cuda.Stream()
    scene.bloom(c, b, out, width=W, height=H, stream=s)  # allocates this key's scratch and plans
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        with pytest.raises(bh.BhError):  # a new size under capture: refused, nothing launched
            scene.bloom(c, b, out, width=W - 8, height=H, stream=s)
        with pytest.raises(bh.BhError):  # the same size with a schedule not run before: refused
            scene.bloom(c, b, out, width=W, height=H, schedule=bh.BH_BLOOM_LITERAL, stream=s)
        scene.bloom(c, b, out, width=W, height=H, stream=s)
    for k in range(bh.BH_BLOOM_SETS + 2):  # other sizes: evict every set no graph holds
        w = W - 8 * (k + 1)
        scene.bloom(c, b, torch.zeros_like(c), width=w, height=H, stream=s)
    torch.cuda.synchronize()
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), oracle.bloom(col, bo, 3))
    del g
    scene.graph_release()
    scene.bloom(c, b, torch.zeros_like(c), width=W - 64, height=H, stream=s)  # may evict it now
    torch.cuda.synchronize()
    scene.close()
