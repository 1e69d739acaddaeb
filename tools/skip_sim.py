"""How often could a march step skip its three SDF square roots?  (diagnostic estimate, CPU, float32 numpy)

A step's dt = min(0.9 * dist, dtm * r) (src/black_hole_maybe.wgsl:299-310) only needs dist when dist
could fall below dtm * r / 0.9, and the surface test only when dist < 0.001.  Root-free sufficient
conditions on the squared arguments the step computes anyway (rho2, y*y, the markers' qm, the photon
sphere's qps) against B = 2 (dtm / 0.9)^2 r2 (with margin) decide "dt == dtm * r, no surface" without
the roots: (a + b)^2 <= 2 a^2 + 2 b^2 gives
    disc:    max(y*y - 2*0.02^2, rho2 - 2*6^2) >= B    or   rho2 <= 9 - 6 * (dtm / 0.9) r
    markers: qm - 2*0.5^2 >= B;   photon sphere: qps - 2*0.075^2 >= B.
A wave skips the roots when every live lane passes.  This script marches a sample of the headline
frame's 8x8 tiles (camera A, 4096x2048, cap 512) in float32 (not the exact arithmetic: an estimate)
and reports the share of wave-steps that would skip, against the share where dt == dtm*r holds exactly.
    python tools/skip_sim.py [--tiles 1024] [--cap 512]"""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import black_hole_ray_marching_amd as bh  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--tiles", type=int, default=1024)
p.add_argument("--cap", type=int, default=512)
p.add_argument("--seed", type=int, default=1)
p.add_argument("--camera", default="0,0,-20")
a = p.parse_args()
W, H = 4096, 2048
f32 = np.float32
cu = bh.CameraUniform()
cu.update(bh.Camera.look_at(tuple(float(v) for v in a.camera.split(",")), (0.0, 0.0, 0.0), W, H))
tri = cu.world_tri.astype(f32)
ro0 = cu.pos.astype(f32)[:3]
rng = np.random.default_rng(a.seed)
tiles = rng.choice((W // 8) * (H // 8), size=a.tiles, replace=False)
tx, ty = tiles % (W // 8), tiles // (W // 8)
lx, ly = np.meshgrid(np.arange(8), np.arange(8))
px = (tx[:, None] * 8 + lx.ravel()[None, :]).ravel().astype(f32)
py = (ty[:, None] * 8 + ly.ravel()[None, :]).ravel().astype(f32)
l0 = (px + f32(0.5)) / f32(2 * W)
l2 = (py + f32(0.5)) / f32(2 * H)
l1 = (f32(1) - l0) - l2
d = l0[:, None] * tri[0] + l1[:, None] * tri[1] + l2[:, None] * tri[2]
rd = (d / np.sqrt((d * d).sum(1, keepdims=True))).astype(f32)
n = rd.shape[0]
ro = np.broadcast_to(ro0, (n, 3)).astype(f32).copy()
h = np.cross(ro, rd).astype(f32)
s = (f32(-1.5) * (h * h).sum(1)).astype(f32)
cps = (-ro0 / np.sqrt((ro0 * ro0).sum()) * f32(1.5)).astype(f32)
trav = np.zeros(n, f32)
live = np.ones(n, bool)
DTM, K = f32(0.5), f32(0.5 / 0.9 * (1 + 2**-15))
C2 = f32(2 * (0.5 / 0.9) ** 2 * (1 + 2**-15))


def accel(p):
    q = (p * p).sum(1)
    return (s / q ** f32(2.5))[:, None] * p


wave_steps = skip_steps = exact_steps = 0
term_combo = {}  # wave-steps that fail the all-terms test: which terms every live lane clears
radius = {"steps": 0, "photon by radius": 0, "markers by radius": 0, "both": 0}  # non-far wave-steps
cond_hits = np.zeros(4)
var_hits = {}
tr_counts = [0, 0]
prev_dec = prev_act = None
for it in range(a.cap):
    lw = live.reshape(-1, 64)
    act = lw.any(1)
    if not act.any():
        break
    r2 = (ro * ro).sum(1)
    r = np.sqrt(r2)
    blackout = ~(r2 > f32(1 + 2**-23))
    x, y, z = ro[:, 0], ro[:, 1], ro[:, 2]
    rho2 = x * x + z * z
    rho = np.sqrt(rho2)
    disc = np.maximum(np.maximum(rho - f32(6), f32(3) - rho), np.abs(y) - f32(0.02))
    yy = y * y
    zz = (f32(-10) - z) ** 2
    q = np.minimum(np.minimum(x * x + (f32(10) - y) ** 2, x * x + (f32(-10) - y) ** 2),
                   np.minimum((f32(10) - x) ** 2 + yy, (f32(-10) - x) ** 2 + yy)) + zz
    m = np.sqrt(q) - f32(0.5)
    ds = np.minimum(disc, m)
    surface = ds < f32(0.001)
    dc = cps - ro
    qps = (dc * dc).sum(1)
    dps = np.sqrt(qps) - f32(0.075)
    dist = np.minimum(ds, dps)
    A = DTM * r
    dt = np.minimum(dist * f32(0.9), A)
    B = C2 * r2
    c_disc = (np.maximum(yy - f32(0.0008 + 1e-6), rho2 - f32(72.001)) >= B) | (rho2 <= f32(9) - f32(6) * K * r)
    c_mark = np.minimum(q - f32(0.5001), qps - f32(0.01126)) >= B
    fast = (c_disc & c_mark) | blackout
    # tight forms: value >= (T + c)^2 with T = K r  (T^2 + 2cT + c^2)
    T = K * r
    th = lambda c: (T + f32(c)) ** 2
    t_y = yy >= th(0.02 + 1e-6)
    t_out = rho2 >= th(6.001)
    t_in = (rho2 <= (f32(3) - T) ** 2 * f32(1 - 1e-6)) & (T < f32(3))
    t_m = q >= th(0.5001)
    t_p = qps >= th(0.07501)
    variants = {"tight all": (t_y | t_out | t_in) & t_m & t_p, "tight y|in, m, p": (t_y | t_in) & t_m & t_p,
                "tight y, m, p": t_y & t_m & t_p, "tight in|out, m, p": (t_in | t_out) & t_m & t_p,
                "tight out, m, p": t_out & t_m & t_p, "tight out|y, m, p": (t_out | t_y) & t_m & t_p,
                "tight out, m; loose p": t_out & t_m & (qps - f32(0.01126) >= B)}
    for Rf in (40.0, 45.0, 50.0):
        variants[f"far r >= {Rf}"] = r2 >= f32(Rf * Rf)
    # per-term radii (bh_host.cpp sdf_term_radii): a wave whose staying lanes all lie beyond the photon sphere's
    # radius, or outside the markers' band, clears that term without forming its argument
    k = 1.1251 * 0.5
    r_ps = 1.01 * (1.5 * 1.0001 + 0.078) / (1 - k)
    r_mo = 1.01 * (10 * np.sqrt(2) + 0.5 + 0.003) / (1 - k)
    r_mi = 0.99 * (10 * np.sqrt(2) - 0.5 - 0.003) / (1 + k)
    far_w = (((r2 >= f32(41.5 ** 2 * 1.0201)) | blackout) | ~live).reshape(-1, 64).all(1)
    nf = act & ~far_w
    ps_w = (((r2 >= f32(r_ps ** 2)) | blackout) | ~live).reshape(-1, 64).all(1)
    m_w = ((((r2 >= f32(r_mo ** 2)) | (r2 <= f32(r_mi ** 2))) | blackout) | ~live).reshape(-1, 64).all(1)
    radius["steps"] += int(nf.sum())
    radius["photon by radius"] += int((nf & ps_w).sum())
    radius["markers by radius"] += int((nf & m_w).sum())
    radius["both"] += int((nf & ps_w & m_w).sum())
    # per-term clearance at wave level (tight forms) on the wave-steps the all-terms test sends to the roots
    okw = lambda v: ((v | blackout) | ~live).reshape(-1, 64).all(1)  # noqa: E731
    D, M, P = okw(t_y | t_out | t_in), okw(t_m), okw(t_p)
    slow = act & ~(D & M & P)
    for key, sel_ in (("disc+markers clear, photon not", D & M & ~P), ("photon clear, disc or markers not", P & ~(D & M)),
                      ("disc clear only", D & ~M & ~P), ("markers clear only", M & ~D & ~P), ("none clear", ~D & ~M & ~P),
                      ("disc+photon clear, markers not", D & P & ~M), ("markers+photon clear, disc not", M & P & ~D)):
        term_combo[key] = term_combo.get(key, 0) + int((slow & sel_).sum())
    term_combo["slow"] = term_combo.get("slow", 0) + int(slow.sum())
    # transitions of the wave-level decision (tight out|y, m, p): after a slow step, how often fast?
    dec = (((variants["tight out|y, m, p"] | blackout) | ~live).reshape(-1, 64).all(1))
    if it > 0:
        tr_counts[0] += int((act & prev_act & ~prev_dec).sum())
        tr_counts[1] += int((act & prev_act & ~prev_dec & dec).sum())
    prev_dec, prev_act = dec, act
    for kv, vv in variants.items():
        lvv = ((vv | blackout) | ~live).reshape(-1, 64).all(1)
        var_hits[kv] = var_hits.get(kv, 0) + int((lvv & act).sum())
    exact = ((dt == A) & ~surface) | blackout
    lf = (fast | ~live).reshape(-1, 64).all(1)
    le = (exact | ~live).reshape(-1, 64).all(1)
    wave_steps += int(act.sum())
    skip_steps += int((lf & act).sum())
    exact_steps += int((le & act).sum())
    # lane view: which condition fails on live non-blackout lanes
    lv = live & ~blackout
    cond_hits += [lv.sum(), (lv & ~c_disc).sum(), (lv & ~c_mark).sum(), (lv & ~(exact)).sum()]
    # the step
    done = blackout | surface
    dtv = dt[:, None]
    k1o, k1d = dtv * rd, dtv * accel(ro)
    k2o, k2d = dtv * (rd + f32(0.5) * k1d), dtv * accel(ro + f32(0.5) * k1o)
    k3o, k3d = dtv * (rd + f32(0.5) * k2d), dtv * accel(ro + f32(0.5) * k2o)
    k4o, k4d = dtv * (rd + k3d), dtv * accel(ro + k3o)
    nro = ro + (k1o + f32(2) * k2o + f32(2) * k3o + k4o) / f32(6)
    nrd = rd + (k1d + f32(2) * k2d + f32(2) * k3d + k4d) / f32(6)
    ntr = trav + dt
    go = live & ~done
    ro = np.where(go[:, None], nro, ro).astype(f32)
    rd = np.where(go[:, None], nrd, rd).astype(f32)
    trav = np.where(go, ntr, trav).astype(f32)
    live = go & ~(ntr > f32(250))
print(f"tiles {a.tiles}, wave-steps {wave_steps}: skippable (root-free test) {skip_steps / wave_steps:.3f}, "
      f"dt == dtm*r and no surface on every lane {exact_steps / wave_steps:.3f}")
print("live lane-steps %d: disc test fails %.3f, marker/photon test fails %.3f, exact condition fails %.3f"
      % (cond_hits[0], cond_hits[1] / cond_hits[0], cond_hits[2] / cond_hits[0], cond_hits[3] / cond_hits[0]))
for kv, vv in var_hits.items():
    print(f"  {kv}: {vv / wave_steps:.3f}")
print(f"after a slow wave-step: {tr_counts[0]} steps, of them fast {tr_counts[1] / max(tr_counts[0], 1):.3f}")
print(f"non-far wave-steps {radius['steps'] / wave_steps:.3f} of all; of them " +
      ", ".join(f"{k} {v / max(radius['steps'], 1):.3f}" for k, v in radius.items() if k != "steps"))
sl = max(term_combo.get("slow", 0), 1)
print(f"wave-steps taking the roots (tight all-terms test fails): {sl / wave_steps:.3f} of all; of them, per term:")
for kv, vv in term_combo.items():
    if kv != "slow":
        print(f"  {kv}: {vv / sl:.3f}")
