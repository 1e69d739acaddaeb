"""Where a march wave's lifetime goes (diagnostic; needs a library built with -DBH_DIAG_PHASES=1, e.g.
`tools/build_variant.sh phases -DBH_DIAG_PHASES=1`, run with BH_LIB=tools/variants/phases.so).

The clock-probed waves (one in `stride`) add the shader cycles of five phases to their XCD's
accumulator (bh_march.hpp, BH_DIAG_PHASES): tables staged, tile + pixel ray, march, shading + store,
cost bookkeeping.  Prints the mean cycles per sampled wave and each phase's share of the lifetime, for
the headline workload (4096x2048, cap 512, camera A, 32 frames per launch, RGBA16F, two targets).
    BH_LIB=tools/variants/phases.so python tools/probe_phases.py [--launches 20]
config 1 (256x256, cap 64, no surfaces, 256 frames per launch):
    ... tools/probe_phases.py --width 256 --height 256 --cap 64 --frames 256 --no-surfaces --stride 4"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import black_hole_ray_marching_amd as bh  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--width", type=int, default=4096)
p.add_argument("--height", type=int, default=2048)
p.add_argument("--cap", type=int, default=512)
p.add_argument("--frames", type=int, default=32)
p.add_argument("--launches", type=int, default=20)
p.add_argument("--stride", type=int, default=64)
p.add_argument("--no-surfaces", action="store_true", help="scene_flags 0 (BASELINE config 1's scene)")
args = p.parse_args()
W, H, D = args.width, args.height, args.frames
scene = bh.Scene(W, H, sky=bh.synthetic_sky(4096, 2048), max_iters=args.cap, math=bh.BH_MATH_EXACT,
                 **(dict(scene_flags=0) if args.no_surfaces else {}))
cols = [torch.empty((H, W, 4), dtype=torch.float16, device="cuda") for _ in range(D)]
bos = [torch.empty((H, W, 4), dtype=torch.float16, device="cuda") for _ in range(D)]
batch = scene.prepare_frames(cols, bos, fmt=bh.BH_OUT_RGBA16F)
for _ in range(5):  # warm-up (clock ramp, learned order)
    batch.render()
torch.cuda.synchronize()
acc = torch.zeros(128, dtype=torch.int64, device="cuda")
scene.set_clock_probe(acc, args.stride)
for _ in range(args.launches):
    batch.render()
torch.cuda.synchronize()
scene.set_clock_probe(None)
a = acc.cpu().numpy().view(np.uint64).reshape(8, 16).astype(np.float64)
waves = a[:, 2].sum()
names = ["tables", "tile+ray", "march", "shade+store", "cost"]
ph = a[:, 3:8].sum(0) / max(waves, 1)
life = a[:, 0].sum() / max(waves, 1)
out = {"waves": int(waves), "mhz": round(float(100.0 * a[:, 0].sum() / max(a[:, 1].sum(), 1)), 1),
       "lifetime_cycles": round(float(life), 1),
       "phases_cycles": {n: round(float(v), 1) for n, v in zip(names, ph)},
       "phases_share": {n: round(float(v / life), 4) for n, v in zip(names, ph)}}
print(json.dumps(out))
scene.close()
