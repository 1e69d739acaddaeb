"""CPU tests of bh_bloom_check: the host-side bound checks of every bloom launch (no GPU needed).

bh_bloom_check plans a chain exactly as bh_bloom does (schedule choice, separable and same-size plans,
every kernel form the launchers pick) and, instead of launching, replays each launch's index arithmetic
on the host: every block's staged footprint inside its LDS tile, every tile read inside the footprint,
every plan index and fix-up list entry inside its texture (DESIGN.md §7b "Bound checks").  Round 4's
GPU memory-access fault (a fix-up launch sized from a freed plan record) is the class of bug these
checks and this sweep exist for; the reference's chain is src/bloom.rs:53-71 and the 8-tap filter
src/kawase_upsample.wgsl:29-39.
"""
import ctypes as C
import os
import subprocess
import sys
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

import pytest

import black_hole_ray_marching_amd as bh
from black_hole_ray_marching_amd import _abi

ROOT = Path(__file__).resolve().parent.parent


def _check(W, H, levels, schedule=bh.BH_BLOOM_AUTO):
    lib = bh.load()
    n = C.c_uint64()
    st = lib.bh_bloom_check(W, H, levels, schedule, C.byref(n), None, 0)
    return st, n.value, (lib.bh_last_error().decode() if st else "")


def _sweep(args):
    """One chunk of the sweep (a worker process): the failures, as (W, H, levels, schedule, message)."""
    sizes, levels, schedule = args
    bad = []
    for W, H in sizes:
        st, n, msg = _check(W, H, levels, schedule)
        if st != 0 or n == 0:
            bad.append((W, H, levels, schedule, msg or f"status {st}, {n} launches"))
    return bad


def _run_sweep(jobs):
    workers = min(8, os.cpu_count() or 1)
    bad = []
    with ProcessPoolExecutor(max_workers=workers) as ex:
        for b in ex.map(_sweep, jobs):
            bad.extend(b)
    return bad


def _chunks(sizes, k=150):
    return [sizes[i:i + k] for i in range(0, len(sizes), k)]


@pytest.mark.parametrize("schedule", [bh.BH_BLOOM_AUTO, bh.BH_BLOOM_LITERAL])
@pytest.mark.parametrize("W,H", [(4096, 2048), (1920, 1080), (1280, 720), (8192, 4096), (2048, 1024), (7, 300),
                                 (300, 7), (1, 1), (1, 2100), (2100, 1), (53, 37),
                                 (2560, 1440), (3840, 2160),
                                 # wider than 2048: same-size copies that are not identities (same_copy passes)
                                 (3440, 1440), (3840, 1080), (2795, 661), (2057, 890), (3121, 1017), (4000, 2200)])
@pytest.mark.parametrize("levels", [1, 2, 3, 4, 5, 12])
def test_reference_sizes_pass_every_bound_check(W, H, levels, schedule):
    st, n, msg = _check(W, H, levels, schedule)
    assert st == 0, msg
    assert n >= 1


def test_every_width_and_height_up_to_2100_at_levels_1_to_5():
    """Each axis 1..2100 against the frame sizes the chain meets in practice on the other axis (the
    checks are per axis: a footprint along x depends only on the x sizes, so this covers every W x H
    for those partners), both schedules, levels 1-5."""
    jobs = []
    for levels in range(1, 6):
        for partner in (1080, 2048):
            jobs += [(c, levels, bh.BH_BLOOM_AUTO) for c in _chunks([(w, partner) for w in range(1, 2101)])]
        for partner in (1920, 4096):
            jobs += [(c, levels, bh.BH_BLOOM_AUTO) for c in _chunks([(partner, h) for h in range(1, 2101)])]
        # the literal pass list at every size (AUTO takes it wherever the fused proofs fail)
        jobs += [(c, levels, bh.BH_BLOOM_LITERAL) for c in _chunks([(w, 720) for w in range(1, 2101, 3)])]
        jobs += [(c, levels, bh.BH_BLOOM_LITERAL) for c in _chunks([(1280, h) for h in range(2, 2101, 3)])]
    bad = _run_sweep(jobs)
    assert not bad, f"{len(bad)} failing sizes, e.g. {bad[:4]}"


def test_small_frames_in_both_axes():
    """Every W x H up to 48 x 48 at levels 1-5: the sizes where the levels' textures reach 1 texel and the
    taps' offsets are many texels wide (the largest footprints per block)."""
    jobs = [([(w, h) for w in range(1, 49) for h in range(1, 49)], lv, s)
            for lv in range(1, 6) for s in (bh.BH_BLOOM_AUTO, bh.BH_BLOOM_LITERAL)]
    bad = _run_sweep([(c, lv, s) for sizes, lv, s in jobs for c in _chunks(sizes, 400)])
    assert not bad, f"{len(bad)} failing sizes, e.g. {bad[:4]}"


@pytest.mark.parametrize("W,H", [(65536, 1000), (65536, 8), (8, 65536), (1000, 65536), (65536, 65536),
                                 (65535, 1080), (65536, 1)])
@pytest.mark.parametrize("schedule", [bh.BH_BLOOM_AUTO, bh.BH_BLOOM_LITERAL])
def test_the_65536_limit_plans_and_passes_the_checks(W, H, schedule):
    """bh_bloom accepts sides up to 65536 (as bh_render).  A shape whose plan the host refuses runs the
    general kernel instead of failing the call (it used to return "invalid value")."""
    st, n, msg = _check(W, H, 3, schedule)
    assert st == 0, msg
    assert n >= 1


def test_arguments_outside_the_contract_are_rejected():
    lib = bh.load()
    for W, H, lv, s in ((0, 8, 3, 0), (8, 0, 3, 0), (65537, 8, 3, 0), (8, 8, 0, 0), (8, 8, 13, 0), (8, 8, 3, 2)):
        assert lib.bh_bloom_check(W, H, lv, s, None, None, 0) == _abi.BH_ERR_INVALID_ARG


def test_the_checks_catch_a_footprint_that_overfills_its_tile():
    """The checks' own negative test: BH_BLOOM_CHECK_SLACK=1 makes every tile one entry smaller in the
    checks, and the chains whose footprints fill their tiles exactly must then be reported (in a child
    process: the hook is read once at load)."""
    code = ("import ctypes as C, black_hole_ray_marching_amd as bh\n"
            "lib = bh.load()\n"
            "bad = [(W, H) for W, H in ((1920, 1080), (1280, 720), (4096, 2048), (7, 300))\n"
            "       if lib.bh_bloom_check(W, H, 3, 0, None, None, 0) != 0]\n"
            "print(len(bad), lib.bh_last_error().decode())\n")
    env = dict(os.environ, BH_BLOOM_CHECK_SLACK="1", BH_NO_TORCH_PRELOAD="1", PYTHONPATH=str(ROOT))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    n, _, msg = r.stdout.strip().partition(" ")
    assert int(n) >= 1, r.stdout
    assert "tile" in msg or "footprint" in msg or "span" in msg, msg


def test_fixup_lane_addresses_stay_inside(tmp_path):
    """The final fix-up pass's global reads lane by lane (tools/bloom_fixup_addr.cpp, a host emulation of
    fixup_gather_kernel<EPI_FINAL> with records and column strips, from the library's own plan builders in
    its bh_bloom.o): every index inside its buffer -- the dead lanes past the list included, whose stale
    column record indexed rows at 3996 x 495 (round 6's GPU memory fault)."""
    obj = ROOT / "black_hole_ray_marching_amd" / "_build" / "bh_bloom.o"
    hipcc = Path(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"))
    if not obj.exists() or not hipcc.exists():
        pytest.skip("needs the built bh_bloom.o and hipcc")
    o, exe = tmp_path / "fa.o", tmp_path / "fa"
    subprocess.run(["g++", "-O2", "-std=c++17", "-c", str(ROOT / "tools" / "bloom_fixup_addr.cpp"), "-o", str(o)], check=True)
    subprocess.run([str(hipcc), "--offload-arch=gfx950", str(o), str(obj), "-o", str(exe)], check=True)
    named = ["3996", "495", "1868", "83", "3840", "2160", "1920", "1080", "1", "1", "4096", "1"]
    r = subprocess.run([str(exe), *named], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:]
    r = subprocess.run([str(exe), "sweep", "150", "6", "4200", "2300"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
