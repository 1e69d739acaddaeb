"""The app's frame as one measured path: State::render = Scene::render (BGRA8, both
targets) + Bloom::render (/root/reference/src/state.rs:270-286), per frame, on one GPU:
  march      bh_render alone (one frame per launch; `batch` frames per bh_render_frames launch when batch > 1)
  bloom      bh_bloom alone
  serial     march then bloom on one stream, frame after frame
  pipelined  bh_presenter (include/bh_render.h): a call's frames march while the previous call's are bloomed on a
             second stream (defaults: 3 calls in flight, march streams auto); variants: `pipelined_d<N>m<K>` N
             calls in flight (target banks) and K march streams (K = 2: the next call's march also starts under this
             one's tail), `pipelined_cus<k>` the bloom on k CUs and the march on the others
`hidden` = (serial - pipelined) / bloom: the share of the bloom the pipeline hides.  HIP events on the caller's
stream around `frames` frames (after a warm-up); the shader clock of the march launches (bh_set_clock_probe)
during the pipelined run; `roofline`: the march's algorithmic FP32 work (the frames' executed-RK-step counts from
the kernel's debug output x 209 flop-eq) per pipelined frame time against 157.3 TFLOP/s.
    python tools/bench_frame.py [--sizes 1280x720:256,1920x1080:256,4096x2048:512] [--camera orbit|A] [--batch 1]"""
import argparse
import json
import math
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import black_hole_ray_marching_amd as bh  # noqa: E402

F_STEP, PEAK = 209.0, 157.3e12
p = argparse.ArgumentParser()
p.add_argument("--sizes", default="1280x720:256,1920x1080:256,4096x2048:512")
p.add_argument("--camera", choices=["orbit", "A", "B"], default="orbit")
p.add_argument("--frames", type=int, default=64)
p.add_argument("--batch", type=int, default=1)
p.add_argument("--cus", default="8", help="comma list of bloom CU counts for the CU-split variant ('' = none)")
p.add_argument("--variants", default="d2m1,d3m1,d3m2",
               help="presenter variants beyond the default (depth 3, march streams auto): dNmK = depth N, K march streams")
p.add_argument("--only-pipelined", action="store_true",
               help="time the default presenter only (a rocprofv3 trace of the pipeline: tools/prof_overlap.py)")
p.add_argument("--no-roofline", action="store_true", help="skip the debug renders that count the executed RK steps")
args = p.parse_args()


def cameras(n, W, H):
    out = []
    for i in range(n):
        cu = bh.CameraUniform()
        if args.camera == "orbit":  # every frame its own camera: a 360-degree orbit at radius 20, 2 above the disc
            a = 2 * math.pi * i / n
            cu.update(bh.Camera.look_at((20 * math.sin(a), 2.0, -20 * math.cos(a)), (0.0, 0.0, 0.0), W, H))
        elif args.camera == "A":
            cu.update(bh.Camera.default(W, H))
        else:
            cu.update(bh.Camera.look_at((0.0, 3.0, -20.0), (0.0, 0.0, 0.0), W, H))
        out.append(cu)
    return out


def timed(fn, stream, n):
    fn(stream, warm=True)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    fn(stream, warm=False)
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


for spec in args.sizes.split(","):
    size, cap = spec.split(":")
    W, H = (int(v) for v in size.split("x"))
    cap = int(cap)
    F, D = args.frames, args.batch
    assert F % D == 0
    scene = bh.Scene(W, H, sky=bh.synthetic_sky(), max_iters=cap, math=bh.BH_MATH_EXACT)
    cams = cameras(F, W, H)
    # the frames' executed RK steps (kernel debug output), for the roofline
    steps = torch.empty((H, W), dtype=torch.int16, device="cuda")
    col = [torch.empty((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(D)]
    bo = [torch.empty_like(col[0]) for _ in range(D)]
    total_steps = 0
    for c in ([] if args.no_roofline else cams):
        scene.camera_uniform = c
        scene.render(col[0], bo[0], fmt=bh.BH_OUT_BGRA8_SRGB, dbg_steps=steps)
        total_steps += int(steps.cpu().numpy().view(np.uint16).astype(np.int64).sum())
    surf = [torch.empty_like(col[0]) for _ in range(F)]
    s = torch.cuda.Stream()
    batch = scene.prepare_frames(col, bo, fmt=bh.BH_OUT_BGRA8_SRGB)

    def march(st, warm):
        for k in range(0, 8 if warm else F, D):
            batch.render(cameras=cams[k:k + D], stream=st)

    def bloom(st, warm):
        for k in range(8 if warm else F):
            scene.bloom(col[k % D], bo[k % D], surf[k], stream=st)

    def serial(st, warm):
        for k in range(0, 8 if warm else F, D):
            batch.render(cameras=cams[k:k + D], stream=st)
            for i in range(D):
                scene.bloom(col[i], bo[i], surf[k + i], stream=st)

    def piped(pr):
        def run(st, warm):
            for k in range(0, 8 if warm else F, D):
                pr.present(surf[k:k + D], cameras=cams[k:k + D], stream=st)
        return run

    row = {"width": W, "height": H, "max_iters": cap, "camera": args.camera, "frames": F, "batch": D}
    if args.only_pipelined:
        pr = bh.Presenter(scene, batch=D)
        row["pipelined_ms"] = round(timed(piped(pr), s, F), 5)
        pr.close()
        print(json.dumps(row), flush=True)
        scene.close()
        continue
    row.update(march_ms=round(timed(march, s, F), 5), bloom_ms=round(timed(bloom, s, F), 5),
               serial_ms=round(timed(serial, s, F), 5))
    # verify: the pipelined surfaces equal the serial ones (the serial run just wrote surf)
    ref = [t.clone() for t in surf]
    pr = bh.Presenter(scene, batch=D)
    acc = torch.zeros(128, dtype=torch.int64, device="cuda")
    scene.set_clock_probe(acc, 64)
    row["pipelined_ms"] = round(timed(piped(pr), s, F), 5)
    scene.set_clock_probe(None)
    torch.cuda.synchronize()
    row["pipelined_equals_serial"] = all(torch.equal(a, b) for a, b in zip(ref, surf))
    row["clock_mhz"] = bh.clock_mhz(acc.cpu().numpy())["mhz"]
    pr.close()
    for v in filter(None, args.variants.split(",")):
        dep, ms = (int(x) for x in v[1:].split("m"))
        pr = bh.Presenter(scene, batch=D, depth=dep, march_streams=ms)
        row[f"pipelined_{v}_ms"] = round(timed(piped(pr), s, F), 5)
        pr.close()
    for k in filter(None, args.cus.split(",")):
        pr = bh.Presenter(scene, batch=D, bloom_cus=int(k))
        row[f"pipelined_cus{k}_ms"] = round(timed(piped(pr), s, F), 5)
        pr.close()
    best = min(v for kk, v in row.items() if kk.startswith("pipelined") and kk.endswith("_ms"))
    row["hidden"] = round((row["serial_ms"] - best) / row["bloom_ms"], 3)
    row["speedup_vs_serial"] = round(row["serial_ms"] / best, 3)
    if args.no_roofline:
        print(json.dumps(row), flush=True)
        scene.close()
        continue
    flop = total_steps / F * F_STEP
    row["roofline"] = {"bound": "valu", "achieved": round(flop / (best * 1e-3) / 1e12, 2), "peak": PEAK / 1e12,
                       "unit": "TFLOP/s", "frac": round(flop / (best * 1e-3) / PEAK, 4),
                       "note": "march work only (executed RK steps x 209 flop-eq) per presented frame"}
    print(json.dumps(row), flush=True)
    scene.close()
