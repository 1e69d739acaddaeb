"""The root-free march step (bh_march.hpp, sdf_skip): a lane that passes the test must have dt == dtm*r and
no surface hit in the full step -- checked here on the step's own float32 arithmetic (numpy: IEEE
add/mul and correctly rounded sqrt, as the exact mode's cores), with samples packed against the test's
thresholds and the dt boundary (src/black_hole_maybe.wgsl:285-310)."""
import numpy as np
import pytest

f32 = np.float32
DISC, MARKERS = 1, 2


def fma32(a, b, c):
    return (a.astype(np.float64) * np.float64(b) + np.float64(c)).astype(f32)


def fms(u, v):
    """fma(-u, u, v): v - u*u rounded once (float64 holds u*u exactly; inf - inf is NaN, as the fma's)"""
    with np.errstate(invalid="ignore", over="ignore"):
        return (v.astype(np.float64) - u.astype(np.float64) ** 2).astype(f32)


def predicate(flags, dtr, rho2, yy, qm, qps, rs):
    """sdf_skip_slack(...) >= 0 (NaN fails)"""
    T = fma32(dtr, 1.125, f32(0.002))
    u6 = T + f32(6.0) * rs
    uy, um, up = T + f32(0.02), T + f32(0.5), T + f32(0.075)
    inf = np.full_like(dtr, np.inf)
    disc = np.fmax(fms(u6, rho2), fms(uy, yy)) if flags & DISC else inf
    mark = fms(um, qm) if flags & MARKERS else inf
    slack = np.fmin(np.fmin(disc, mark), fms(up, qps))
    return slack >= 0


def full_step(flags, dtr, rho2, y, qm, qps, rs):
    """dt and the surface test of the full step (the exact mode's op sequence)."""
    rho = np.sqrt(rho2)
    disc = np.fmax(np.fmax(rho - f32(6.0) * rs, -(rho - f32(3.0) * rs)), np.abs(y) - f32(0.02))
    m = np.sqrt(qm) - f32(0.5)
    inf = f32(np.inf)
    ds = np.fmin(disc if flags & DISC else inf, m if flags & MARKERS else inf)
    dps = np.sqrt(qps) - f32(0.075)
    dist = np.fmin(ds, dps)
    dt = np.fmin(dist * f32(0.9), dtr)
    return dt, ds < f32(0.001)


def samples(rng, n, rs, dtm):
    r = np.exp(rng.uniform(np.log(1.0), np.log(300.0), n)).astype(f32)
    dtr = (f32(dtm) * r).astype(f32)
    T = fma32(dtr, 1.125, f32(0.002))
    # each distance term sits near its threshold (s ~ 1) or well inside (s ~ 0.5 .. 3)
    def near(c):
        s = np.where(rng.random(n) < 0.7, rng.uniform(0.9995, 1.0005, n), rng.uniform(0.5, 3.0, n))
        return ((T.astype(np.float64) * s + c) ** 2).astype(f32)
    rho2 = np.where(rng.random(n) < 0.5, near(6.0 * rs), rng.uniform(0, 40, n).astype(f32) ** 2).astype(f32)
    y = np.sqrt(near(0.02).astype(np.float64)).astype(f32) * np.where(rng.random(n) < 0.5, f32(1), f32(-1))
    y = np.where(rng.random(n) < 0.3, rng.uniform(-1, 1, n).astype(f32), y).astype(f32)
    qm, qps = near(0.5), near(0.075)
    # single-ulp nudges either way around the thresholds
    for a in (rho2, qm, qps):
        k = rng.integers(-3, 4, n).astype(np.int32)
        a.view(np.int32)[:] += k
    return dtr, rho2, y, qm, qps


@pytest.mark.parametrize("flags", [DISC | MARKERS, DISC, MARKERS])
@pytest.mark.parametrize("rs,dtm", [(1.0, 0.5), (8.0, 0.5), (0.25, 0.01), (1.0, 3.0)])
def test_skip_implies_dt_equals_dtm_r(flags, rs, dtm):
    rng = np.random.default_rng(hash((flags, rs, dtm)) & 0xFFFFFFFF)
    rs = f32(rs)
    passed = 0
    for _ in range(3):
        dtr, rho2, y, qm, qps = samples(rng, 200_000, rs, dtm)
        ok = predicate(flags, dtr, rho2, (y * y).astype(f32), qm, qps, rs)
        dt, surface = full_step(flags, dtr, rho2, y, qm, qps, rs)
        bad = ok & ((dt != dtr) | surface)
        assert not bad.any(), (dtr[bad][:4], rho2[bad][:4], y[bad][:4], qm[bad][:4], qps[bad][:4])
        passed += int(ok.sum())
    assert passed > 50_000  # the samples do exercise the skip


def term_slacks(flags, dtr, rho2, yy, qm, qps, rs):
    """sdf_term_slacks: the disc, marker and photon-sphere terms of the test, each on its own"""
    T = fma32(dtr, 1.125, f32(0.002))
    u6 = T + f32(6.0) * rs
    uy, um, up = T + f32(0.02), T + f32(0.5), T + f32(0.075)
    inf = np.full_like(dtr, np.inf)
    disc = np.fmax(fms(u6, rho2), fms(uy, yy)) if flags & DISC else inf
    mark = fms(um, qm) if flags & MARKERS else inf
    return disc, mark, fms(up, qps)


def step_without(flags, dtr, rho2, y, qm, qps, rs, skip_d, skip_m, skip_p):
    """the per-term step (bh_march.hpp, BH_SDF_TERMS): a left-out term enters dist as +inf"""
    rho = np.sqrt(rho2)
    inf = f32(np.inf)
    disc = np.where(skip_d, inf, np.fmax(np.fmax(rho - f32(6.0) * rs, -(rho - f32(3.0) * rs)), np.abs(y) - f32(0.02)))
    m = np.where(skip_m, inf, np.sqrt(qm) - f32(0.5))
    ds = np.fmin(disc if flags & DISC else inf, m if flags & MARKERS else inf)
    dps = np.where(skip_p, inf, np.sqrt(qps) - f32(0.075))
    dt = np.fmin(np.fmin(ds, dps) * f32(0.9), dtr)
    return dt, ds < f32(0.001)


@pytest.mark.parametrize("flags", [DISC | MARKERS, DISC, MARKERS])
@pytest.mark.parametrize("rs,dtm", [(1.0, 0.5), (8.0, 0.5), (0.25, 0.01), (1.0, 3.0)])
def test_per_term_skip_keeps_dt_and_surface(flags, rs, dtm):
    """Any subset of the terms whose own slack holds may be left out of dist: the step's dt and surface
    test are those of the full step, bit for bit (the wave leaves out a term only where every lane that
    stays clears it, so a lane's left-out terms are always a subset of its cleared ones)."""
    rng = np.random.default_rng(hash((flags, rs, dtm, "terms")) & 0xFFFFFFFF)
    rs = f32(rs)
    cleared = 0
    for _ in range(1):
        dtr, rho2, y, qm, qps = samples(rng, 150_000, rs, dtm)
        yy = (y * y).astype(f32)
        sd, sm, sp = term_slacks(flags, dtr, rho2, yy, qm, qps, rs)
        cd, cm, cp = sd >= 0, sm >= 0, sp >= 0
        dt, surface = full_step(flags, dtr, rho2, y, qm, qps, rs)
        for mask in range(1, 8):
            skip_d = cd & bool(mask & 1)
            skip_m = cm & bool(mask & 2)
            skip_p = cp & bool(mask & 4)
            dt2, surface2 = step_without(flags, dtr, rho2, y, qm, qps, rs, skip_d, skip_m, skip_p)
            bad = (dt2.view(np.int32) != dt.view(np.int32)) | (surface2 != surface)
            assert not bad.any(), (mask, dtr[bad][:4], rho2[bad][:4], y[bad][:4], qm[bad][:4], qps[bad][:4])
        cleared += int((cd | cm | cp).sum())
    assert cleared > 50_000


def test_skip_rejects_nan_and_infinite_thresholds():
    rs = f32(1.0)
    dtr = np.array([0.5, np.nan, 0.5, 0.5, np.inf, np.inf], f32)
    big = np.array([np.inf, 1e6, np.nan, 1e6, 1e6, np.inf], f32)
    ok = predicate(DISC | MARKERS, dtr, big, big, big, big, rs)
    assert ok.tolist() == [True, False, False, True, False, False]
    dt, surface = full_step(DISC | MARKERS, dtr[[0]], big[[0]], np.sqrt(big[[0]]), big[[0]], big[[0]], rs)
    assert dt[0] == dtr[0] and not surface[0]


def far_r2(rs, dtm):
    """mirror of bh_host.cpp sdf_far_r2"""
    k = 1.1251 * dtm
    a1, a2 = np.sqrt(0.5) - k, 1.0 - k
    if not a1 > 0.01:
        return np.inf
    R0 = max((max(6.0 * rs, 0.02) + 0.003) / a1, (10.0 * np.sqrt(2.0) + 0.5 + 0.003) / a2, (1.5 * rs + 0.075 + 0.003) / a2)
    return np.nextafter(f32((1.01 * R0) ** 2), f32(np.inf))


def step_from_point(p, rs, dtm, cam):
    """dt and the surface test of the full step at positions p (n, 3) float32 -- the exact mode's op
    sequence from the position itself (bh_march.hpp sdf_args / sdf_from, :285-310)."""
    x, y, z = p[:, 0], p[:, 1], p[:, 2]
    r2 = (x * x + y * y) + z * z
    r = np.sqrt(r2)
    dtr = f32(dtm) * r
    rho = np.sqrt(x * x + z * z)
    disc = np.fmax(np.fmax(rho - f32(6.0) * rs, -(rho - f32(3.0) * rs)), np.abs(y) - f32(0.02))
    zz = (f32(-10.0) - z) ** 2
    ty, tx = f32(10.0) - np.abs(y), f32(10.0) - np.abs(x)
    qm = np.fmin((x * x + ty * ty) + zz, (tx * tx + y * y) + zz)
    m = np.sqrt(qm) - f32(0.5)
    cps = (-cam / np.sqrt((cam * cam).sum()) * f32(1.5) * rs).astype(f32)
    dc = cps - p
    dps = np.sqrt((dc[:, 0] * dc[:, 0] + dc[:, 1] * dc[:, 1]) + dc[:, 2] * dc[:, 2]) - f32(0.075)
    ds = np.fmin(disc, m)
    dt = np.fmin(np.fmin(ds, dps) * f32(0.9), dtr)
    return r2, dtr, dt, ds < f32(0.001)


@pytest.mark.parametrize("rs,dtm", [(1.0, 0.5), (0.25, 0.5), (8.0, 0.5), (1.0, 0.1), (1.0, 0.6), (0.003, 0.3)])
def test_far_field_implies_dt_equals_dtm_r(rs, dtm):
    """bh_march.hpp's far-field level: every lane with far_r2 <= r^2 <= FLT_MAX has dt == RN(dtm r) and no
    surface hit, checked on points just beyond the radius (all directions, the markers' and the disc plane's
    included) and far out."""
    rng = np.random.default_rng(int(rs * 1000 + dtm * 10))
    F = far_r2(rs, dtm)
    assert np.isfinite(F)
    rs = f32(rs)
    R = np.sqrt(np.float64(F))
    n = 400_000
    d = rng.normal(size=(n, 3))
    d[: n // 4, 1] *= 1e-3               # near the disc plane
    d[n // 4: n // 2] = [0.0, 1.0, -1.0] + 0.02 * rng.normal(size=(n // 4, 3))  # towards a marker
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    mag = np.where(rng.random(n) < 0.8, R * (1 + rng.uniform(0, 1e-3, n)), R * np.exp(rng.uniform(0, 8, n)))
    p = (d * mag[:, None]).astype(f32)
    cam = np.array([0.0, 0.0, -20.0], f32) if rs != f32(8.0) else np.array([3.0, 1.0, -40.0], f32)
    r2, dtr, dt, surface = step_from_point(p, rs, dtm, cam)
    far = (r2 >= F) & (r2 <= f32(np.finfo(np.float32).max))
    assert far.sum() > n // 2
    bad = far & ((dt != dtr) | surface)
    assert not bad.any(), p[bad][:4]


def test_far_field_off_for_large_dtm():
    assert far_r2(1.0, 0.7) == np.inf
