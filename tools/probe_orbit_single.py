"""Why is one frame per launch with a moving camera (bench.py's single_frame_orbit, 0.62 ms) slower than the
fixed camera (single_frame, 0.55 ms)?  For camera A orbiting the hole at `--deg` per frame from `--start`:
  moving     each angle rendered once, in order (the dispatch order learned from the previous angle's frame)
  repeated   each angle rendered three times, the third timed (the order learned from the same camera)
per exact build (auto, issue-order, latency), ms per frame from HIP events around each launch, plus the frames'
capped-ray counts (fate CAP) -- so the gap splits into the scene's own cost at those angles and the order's
staleness.
    python tools/probe_orbit_single.py [--start 20 --deg 0.2 --frames 24]"""
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
p.add_argument("--start", type=float, default=20.0)
p.add_argument("--deg", type=float, default=0.2)
p.add_argument("--frames", type=int, default=24)
p.add_argument("--max-iters", type=int, default=512)
args = p.parse_args()
W, H = 4096, 2048
scene = bh.Scene(W, H, sky=bh.synthetic_sky(), max_iters=args.max_iters, math=bh.BH_MATH_EXACT)
col = torch.empty((H, W, 4), dtype=torch.float16, device="cuda")
bo = torch.empty_like(col)
fate = torch.empty((H, W), dtype=torch.uint8, device="cuda")
pos0, tgt = CAMERAS["A"]


def cam_at(deg):
    a = math.radians(deg)
    x, y, z = pos0
    c = bh.CameraUniform()
    c.update(bh.Camera.look_at((x * math.cos(a) + z * math.sin(a), y, -x * math.sin(a) + z * math.cos(a)), tgt, W, H))
    return c


angles = [args.start + k * args.deg for k in range(args.frames)]
cams = [cam_at(d) for d in angles]
builds = {"auto": 0, "issue_order": bh.BH_SCHED_FLAG_ISSUE_ORDER, "latency": bh.BH_SCHED_FLAG_LATENCY}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]


def timed(c, flag):
    batch = scene.prepare_frames([col], [bo], fmt=bh.BH_OUT_RGBA16F, schedule=flag)
    ev[0].record()
    batch.render(cameras=[c])
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1])


capped = []
for c in cams:
    scene.camera_uniform = c
    scene.render(col, bo, fmt=bh.BH_OUT_RGBA16F, dbg_fate=fate)
    torch.cuda.synchronize()
    capped.append(int((fate.cpu().numpy() == 0).sum()))
row = {"start_deg": args.start, "deg_per_frame": args.deg, "frames": args.frames, "max_iters": args.max_iters,
       "capped_mean": round(float(np.mean(capped)), 1), "capped_camera_A": None}
scene.camera_uniform = cam_at(0.0)
scene.render(col, bo, fmt=bh.BH_OUT_RGBA16F, dbg_fate=fate)
torch.cuda.synchronize()
row["capped_camera_A"] = int((fate.cpu().numpy() == 0).sum())
for name, flag in builds.items():
    for _ in range(3):  # warm
        timed(cams[0], flag)
    fixed = [timed(cam_at(0.0), flag) for _ in range(8)][2:]
    moving = [timed(c, flag) for c in cams]
    rep = []
    for c in cams:
        timed(c, flag)
        timed(c, flag)
        rep.append(timed(c, flag))
    row[name] = {"fixed_A_ms": round(float(np.mean(fixed)), 4), "moving_ms": round(float(np.mean(moving[1:])), 4),
                 "repeated_ms": round(float(np.mean(rep)), 4)}
print(json.dumps(row), flush=True)
