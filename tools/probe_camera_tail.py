"""Why does a one-frame launch of camera B cost twice camera A's (4096x2048 cap 512: 1.28 vs 0.62 ms)?
Per camera: ms per frame at 1 and 32 frames per launch for each exact build (the source-order one, which
bh_render picks for a throughput-bound frame, and the machine-scheduled one, whose lone tail waves step
faster), and the frame's executed-step statistics (dbg_steps: the cycle fast-forward skips steps n_rk counts).
    python tools/probe_camera_tail.py [--cameras A,B,C --width 4096 --height 2048 --max-iters 512]"""
import argparse
import json
import math
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import black_hole_ray_marching_amd as bh  # noqa: E402
from bench import CAMERAS  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--cameras", default="A,B,C")
p.add_argument("--width", type=int, default=4096)
p.add_argument("--height", type=int, default=2048)
p.add_argument("--max-iters", type=int, default=512)
p.add_argument("--reps", type=int, default=16)
args = p.parse_args()
W, H = args.width, args.height
scene = bh.Scene(W, H, sky=bh.synthetic_sky(), max_iters=args.max_iters, math=bh.BH_MATH_EXACT)
D = 32
outs = [torch.empty((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(D)]
bos = [torch.empty_like(outs[0]) for _ in range(D)]
n_rk = torch.empty((H, W), dtype=torch.int16, device="cuda")
steps = torch.empty_like(n_rk)
fate = torch.empty((H, W), dtype=torch.uint8, device="cuda")
builds = {"issue_order": bh.BH_SCHED_FLAG_ISSUE_ORDER, "latency": bh.BH_SCHED_FLAG_LATENCY, "auto": 0}
for cam in args.cameras.split(","):
    pos, tgt = CAMERAS[cam]
    scene.update(bh.Camera.look_at(pos, tgt, W, H))
    row = {"camera": cam, "width": W, "height": H, "max_iters": args.max_iters}
    scene.render(outs[0], bos[0], fmt=bh.BH_OUT_BGRA8_SRGB, dbg_n_rk=n_rk, dbg_fate=fate, dbg_steps=steps)
    torch.cuda.synchronize()
    nr = n_rk.cpu().numpy().view(np.uint16).astype(np.int64)
    st = steps.cpu().numpy().view(np.uint16).astype(np.int64)
    fa = fate.cpu().numpy()
    tiles = st[: H // 8 * 8, : W // 8 * 8].reshape(H // 8, 8, W // 8, 8).max(axis=(1, 3))
    row.update(capped=int((fa == 0).sum()), capped_full_steps=int(((fa == 0) & (st >= args.max_iters)).sum()),
               mean_n_rk=round(float(nr.mean()), 3), mean_steps=round(float(st.mean()), 3),
               tiles_steps_ge_256=int((tiles >= 256).sum()), tiles_steps_ge_128=int((tiles >= 128).sum()),
               max_steps=int(st.max()))
    for bname, flag in builds.items():
        for per in (1, D):
            batch = scene.prepare_frames(outs[:per], bos[:per], fmt=bh.BH_OUT_BGRA8_SRGB, schedule=flag)
            for _ in range(3):
                batch.render()
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            n = max(1, args.reps * D // per // 4) if per > 1 else args.reps
            ev[0].record()
            for _ in range(n):
                batch.render()
            ev[1].record()
            torch.cuda.synchronize()
            row[f"{bname}_D{per}_ms"] = round(ev[0].elapsed_time(ev[1]) / (n * per), 5)
    print(json.dumps(row), flush=True)
