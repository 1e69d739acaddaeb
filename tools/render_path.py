"""Offline multi-frame render along a scripted camera path: the reference's
frame (Scene::render into the two Bgra8UnormSrgb targets, then Bloom::render) per frame, the camera
driven by CameraController with a key script, PNG frames out.

    python tools/render_path.py --width 1024 --height 512 --frames 24 --dt 0.05 \\
        --script "W:0-12,ArrowLeft:6-24,P:12-18" --out gpurun_out/path
Script: comma-separated KEY:first-last frame ranges (keys held down), reference key names (W A S D
Space F ArrowUp/Down/Left/Right P O)."""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import black_hole_ray_marching_amd as bh  # noqa: E402
from black_hole_ray_marching_amd.png import write_png  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--width", type=int, default=1024)
p.add_argument("--height", type=int, default=512)
p.add_argument("--frames", type=int, default=24)
p.add_argument("--dt", type=float, default=0.05)
p.add_argument("--max-iters", type=int, default=512)
p.add_argument("--script", default="W:0-12,ArrowLeft:6-24,P:12-18")
p.add_argument("--out", default="gpurun_out/path")
p.add_argument("--no-png", action="store_true")
p.add_argument("--sky", default=None, help="image file for the sky (e.g. the reference's space_4096x2048.jpg); "
                                            "default: the synthetic sky")
args = p.parse_args()
W, H = args.width, args.height
keys = []
for item in filter(None, args.script.split(",")):
    k, rng = item.split(":")
    a, b = (int(v) for v in rng.split("-"))
    keys.append((k, a, b))
out_dir = Path(args.out)
out_dir.mkdir(parents=True, exist_ok=True)
sky = bh.load_sky(args.sky) if args.sky else bh.synthetic_sky()
scene = bh.Scene(W, H, sky=sky, max_iters=args.max_iters, math=bh.BH_MATH_EXACT)
ctrl = bh.CameraController()
cam = bh.Camera.default(W, H)
col = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
bo = torch.empty_like(col)
surf = torch.empty_like(col)
log = []
t0 = time.perf_counter()
for f in range(args.frames):
    for k, a, b in keys:
        ctrl.process_key(k, a <= f <= b)
    cam, moved = ctrl.update_camera(cam, args.dt)
    scene.update(cam)
    scene.render(col, bo, fmt=bh.BH_OUT_BGRA8_SRGB)
    scene.bloom(col, bo, surf)
    if not args.no_png:
        write_png(out_dir / f"frame_{f:04d}.png", surf.cpu().numpy())
    log.append({"frame": f, "pos": cam.pos, "dir": cam.dir, "moved": moved})
torch.cuda.synchronize()
dt = time.perf_counter() - t0
(out_dir / "path.json").write_text(json.dumps(log, indent=0))
print(json.dumps({"frames": args.frames, "width": W, "height": H, "seconds": round(dt, 3),
                  "frames_per_s_incl_png": round(args.frames / dt, 2), "out": str(out_dir)}))
