"""Probe: can the Kawase bloom of frame i overlap the march of frame i+1 on one GPU?

The app's frame is Scene::render then Bloom::render (/root/reference/src/state.rs:270-286).  This probe
times, per frame, at one size:
  march     : bh_render (BGRA8, both targets) alone, one frame per launch
  bloom     : bh_bloom alone
  serial    : render(i); bloom(i) on one stream
  pipe:<v>  : render(i) on stream M into ring slot i % R, bloom(i) on stream B after it, render(i + R) waits
              for bloom(i) -- variants <v> of the two streams: priorities and CU masks
              (hipExtStreamCreateWithCUMask)
Cameras orbit (every frame differs).  Prints one JSON line per variant.
    python tools/probe_overlap.py --width 1920 --height 1080 --max-iters 256
"""
import argparse
import ctypes as C
import json
import math
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import black_hole_ray_marching_amd as bh  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--width", type=int, default=1920)
p.add_argument("--height", type=int, default=1080)
p.add_argument("--max-iters", type=int, default=256)
p.add_argument("--frames", type=int, default=64)
p.add_argument("--ring", type=int, default=3)
p.add_argument("--variants", default="all")
p.add_argument("--camera", choices=["orbit", "A", "B"], default="orbit",
               help="orbit: every frame a different camera on a circle of radius 20 looking at the origin")
p.add_argument("--only-march", action="store_true", help="time the march alone (one frame per launch) and exit")
args = p.parse_args()
W, H, F, R = args.width, args.height, args.frames, args.ring

hip = C.CDLL("libamdhip64.so")
hip.hipExtStreamCreateWithCUMask.argtypes = [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(C.c_uint32)]
hip.hipStreamCreateWithPriority.argtypes = [C.POINTER(C.c_void_p), C.c_uint, C.c_int]
hip.hipDeviceGetStreamPriorityRange.argtypes = [C.POINTER(C.c_int), C.POINTER(C.c_int)]
lo, hi = C.c_int(), C.c_int()
hip.hipDeviceGetStreamPriorityRange(C.byref(lo), C.byref(hi))
n_cu = torch.cuda.get_device_properties(0).multi_processor_count


def mk_stream(mask_bits=None, prio=None):
    s = C.c_void_p()
    if mask_bits is not None:
        words = (C.c_uint32 * ((n_cu + 31) // 32))()
        for b in mask_bits:
            words[b // 32] |= 1 << (b % 32)
        rc = hip.hipExtStreamCreateWithCUMask(C.byref(s), len(words), words)
    else:
        rc = hip.hipStreamCreateWithPriority(C.byref(s), 0, {"high": hi.value, "low": lo.value}.get(prio, 0))
    assert rc == 0, rc
    return s.value


scene = bh.Scene(W, H, sky=bh.synthetic_sky(), max_iters=args.max_iters, math=bh.BH_MATH_EXACT)
cams = []
for i in range(F):
    a = 2 * math.pi * i / F
    c = bh.CameraUniform()
    if args.camera == "orbit":
        c.update(bh.Camera.look_at((20 * math.sin(a), 2.0, -20 * math.cos(a)), (0.0, 0.0, 0.0), W, H))
    elif args.camera == "A":
        c.update(bh.Camera.default(W, H))
    else:
        c.update(bh.Camera.look_at((0.0, 3.0, -20.0), (0.0, 0.0, 0.0), W, H))
    cams.append(c)
col = [torch.empty((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(R)]
bo = [torch.empty_like(col[0]) for _ in range(R)]
out = [torch.empty_like(col[0]) for _ in range(R)]


def render(i, s):
    scene.camera_uniform = cams[i]
    scene.render(col[i % R], bo[i % R], fmt=bh.BH_OUT_BGRA8_SRGB, stream=s)


def bloom(i, s):
    scene.bloom(col[i % R], bo[i % R], out[i % R], stream=s)


def timed(fn):
    fn(min(F, 8))  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(F)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / F


base = torch.cuda.current_stream()


def run_march(n):
    for i in range(n):
        render(i, base)


def run_bloom(n):
    for i in range(n):
        bloom(i, base)


def run_serial(n):
    for i in range(n):
        render(i, base)
        bloom(i, base)


def pipe(sm, sb):
    """sm: one march stream or a list (frame i marches on sm[i % len])"""
    sms = sm if isinstance(sm, list) else [sm]
    tms, tb = [torch.cuda.ExternalStream(x) for x in sms], torch.cuda.ExternalStream(sb)

    def run(n):
        done = [None] * n
        for i in range(n):
            tm, smi = tms[i % len(sms)], sms[i % len(sms)]
            if i >= R:
                tm.wait_event(done[i - R])
            render(i, smi)
            e = torch.cuda.Event()
            e.record(tm)
            tb.wait_event(e)
            bloom(i, sb)
            done[i] = torch.cuda.Event()
            done[i].record(tb)
    return run


res = {"width": W, "height": H, "max_iters": args.max_iters, "frames": F, "ring": R, "n_cu": n_cu,
       "prio_range": [lo.value, hi.value]}
res["march"] = timed(run_march)
t0 = time.perf_counter()
run_march(F)
res["march_enqueue"] = (time.perf_counter() - t0) * 1e3 / F  # host time per frame to enqueue (no sync)
torch.cuda.synchronize()
if args.only_march:
    print(json.dumps({k: (round(v, 5) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
    sys.exit(0)
res["bloom"] = timed(run_bloom)
res["serial"] = timed(run_serial)
variants = {
    "normal": lambda: (mk_stream(), mk_stream()),
    "bloom_high": lambda: (mk_stream(), mk_stream(prio="high")),
    "bloom_low": lambda: (mk_stream(), mk_stream(prio="low")),
    "march_high": lambda: (mk_stream(prio="high"), mk_stream()),
    "2march_normal": lambda: ([mk_stream(), mk_stream()], mk_stream()),
    "2march_bloom_high": lambda: ([mk_stream(), mk_stream()], mk_stream(prio="high")),
    "2march_bloom_low": lambda: ([mk_stream(), mk_stream()], mk_stream(prio="low")),
    "2march_march_high": lambda: ([mk_stream(prio="high"), mk_stream(prio="high")], mk_stream()),
}
for k in (8, 16, 32, 64) if args.variants == "all" else ():
    # k CUs for the bloom: every (n_cu / k)-th CU, whatever the bit -> XCD mapping
    step = n_cu // k
    bl = [i * step for i in range(k)]
    mr = [i for i in range(n_cu) if i not in set(bl)]
    variants[f"mask{k}_split"] = (lambda bl=bl, mr=mr: (mk_stream(mr), mk_stream(bl)))
    variants[f"mask{k}_bloomonly"] = (lambda bl=bl: (mk_stream(), mk_stream(bl)))
    variants[f"mask{k}_bloomall_marchrest"] = (lambda mr=mr: (mk_stream(mr), mk_stream(prio="high")))
for name, mk in variants.items():
    if args.variants != "all" and name not in args.variants.split(","):
        continue
    sm, sb = mk()
    res[f"pipe:{name}"] = timed(pipe(sm, sb))
    print(json.dumps({"variant": name, "ms_per_frame": round(res[f"pipe:{name}"], 5)}), flush=True)
# correctness: the pipelined frames equal the serial ones
pipe(mk_stream(), mk_stream(prio="high"))(R)
torch.cuda.synchronize()
got = [o.clone() for o in out]
run_serial(R)
torch.cuda.synchronize()
res["pipe_equals_serial"] = all(torch.equal(a, b) for a, b in zip(got, out))
print(json.dumps({k: (round(v, 5) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
