"""Per-tile work distribution of one frame (the tail analysis of DESIGN.md §5):
    python tools/tail_stats.py [--cap 1000] [--camera A|B|C] [--math exact|fast]
Prints the executed-step histogram of tiles' slowest rays and the kernel time."""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import black_hole_ray_marching_amd as bh  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--cap", type=int, default=1000)
p.add_argument("--camera", default="A")
p.add_argument("--math", default="exact")
args = p.parse_args()
W, H = 4096, 2048
cams = {"B": ((0.0, 3.0, -20.0), (0.0, 0.0, 0.0)), "C": ((0.0, 6.0, -12.0), (0.0, 0.0, 0.0))}
sc = bh.Scene(W, H, sky=bh.synthetic_sky(), max_iters=args.cap,
              math=bh.BH_MATH_EXACT if args.math == "exact" else bh.BH_MATH_FAST)
if args.camera != "A":
    sc.update(bh.Camera.look_at(*cams[args.camera], W, H))
col = torch.empty((H, W, 4), dtype=torch.float16, device="cuda")
bo = torch.empty_like(col)
steps = torch.zeros((H, W), dtype=torch.int16, device="cuda")
nrk = torch.zeros((H, W), dtype=torch.int16, device="cuda")
for _ in range(5):
    sc.render(col, bo, fmt=bh.BH_OUT_RGBA16F)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ts = []
for _ in range(20):
    ev[0].record(); sc.render(col, bo, fmt=bh.BH_OUT_RGBA16F); ev[1].record(); torch.cuda.synchronize()
    ts.append(ev[0].elapsed_time(ev[1]))
sc.render(col, bo, fmt=bh.BH_OUT_RGBA16F, dbg_steps=steps, dbg_n_rk=nrk)
torch.cuda.synchronize()
s = steps.cpu().numpy().view(np.uint16).astype(np.int64)
n = nrk.cpu().numpy().view(np.uint16).astype(np.int64)
tmax = s.reshape(H // 8, 8, W // 8, 8).max(axis=(1, 3))
print(f"kernel avg {np.mean(ts):.4f} ms min {np.min(ts):.4f}; sum n_rk {n.sum()} sum steps {s.sum()}; "
      f"rays at cap {(n >= args.cap).sum()}, of them fast-forwarded {((n >= args.cap) & (s < n)).sum()}")
edges = [0, 16, 32, 64, 128, 256, 512, 768, 1000, 100000]
h, _ = np.histogram(tmax, bins=edges)
print("tiles by slowest ray's executed steps:", dict(zip([f"{a}-{b}" for a, b in zip(edges, edges[1:])], h.tolist())))
print("top tile max steps:", np.sort(tmax.ravel())[-10:])
ws = tmax.sum()
print(f"wave-steps {ws} (mean {tmax.mean():.2f} per tile); beyond {48} iterations: {np.maximum(tmax - 48, 0).sum()} "
      f"({np.maximum(tmax - 48, 0).sum() / ws:.1%}) in {(tmax > 48).sum()} tiles; lane-steps / (64 x wave-steps) = "
      f"{s.sum() / (64 * ws):.3f}")
