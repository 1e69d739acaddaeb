"""Which part of a frame slows down after the GPU idles (VERDICT r01 "Next round" 6)?  For each variant:
1 s idle, then K frames (one launch each, HIP events); prints the mean of frames 2-6 over the mean of
the last 10.  The shader clock is flat within 3 % from the first frame after idle
(tools/clock_series.py), so a ratio well above that points at another resource.

    python tools/ramp_probe.py [--frames 50]"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=50)
    a = p.parse_args()
    import torch
    import black_hole_ray_marching_amd as bh
    sky = bh.synthetic_sky()
    W, H = 4096, 2048
    c16 = torch.empty((H, W, 4), dtype=torch.float16, device="cuda")
    b16 = torch.empty_like(c16)
    c8 = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    b8 = torch.empty_like(c8)
    big = torch.empty((4 * H * W * 8,), dtype=torch.uint8, device="cuda")  # 268 MB

    def frames(fn, k):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
        for s, e in ev:
            s.record()
            fn()
            e.record()
        torch.cuda.synchronize()
        return [s.elapsed_time(e) for s, e in ev]

    def scene_fn(cap=512, math=bh.BH_MATH_EXACT, fmt=bh.BH_OUT_RGBA16F, two=True, sched=0, flags=bh.BH_SCENE_DEFAULT):
        sc = bh.Scene(W, H, sky=sky, max_iters=cap, math=math, scene_flags=flags)
        c, b = (c16, b16) if fmt == bh.BH_OUT_RGBA16F else (c8, b8)
        return sc, lambda: sc.render(c, b if two else None, fmt=fmt, schedule=bh.BH_SCHED_TILE | sched)

    variants = {
        "default": dict(),
        "fast_math": dict(math=bh.BH_MATH_FAST),
        "bgra8": dict(fmt=bh.BH_OUT_BGRA8_SRGB),
        "col_only": dict(two=False),
        "cap64": dict(cap=64),
        "no_surfaces": dict(flags=0),
        "latency_build": dict(sched=bh.BH_SCHED_FLAG_LATENCY),
    }
    out = {}
    for name, kw in variants.items():
        sc, fn = scene_fn(**kw)
        fn()
        torch.cuda.synchronize()
        time.sleep(1.0)
        t = frames(fn, a.frames)
        sc.close()
        out[name] = {"first": round(sum(t[1:6]) / 5, 4), "last": round(sum(t[-10:]) / 10, 4),
                     "ratio": round(sum(t[1:6]) / 5 / (sum(t[-10:]) / 10), 4), "ms": [round(x, 4) for x in t]}
        print(name, out[name]["first"], out[name]["last"], out[name]["ratio"], flush=True)
    time.sleep(1.0)
    t = frames(lambda: big.fill_(1), a.frames)
    out["fill_268MB"] = {"first": round(sum(t[1:6]) / 5, 4), "last": round(sum(t[-10:]) / 10, 4),
                         "ratio": round(sum(t[1:6]) / 5 / (sum(t[-10:]) / 10), 4)}
    print("fill_268MB", out["fill_268MB"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
