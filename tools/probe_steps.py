"""Where a frame's executed RK steps go, per 8x8 tile (one wave of the tile schedule): renders a
configuration a few times (so the temporal order is learned) with the debug outputs, then reports
the per-tile maximum of EXECUTED steps (dbg_steps: the cycle fast-forward skips steps that n_rk still
counts) against the normative n_rk, and saves the per-pixel arrays for offline analysis.

    python tools/probe_steps.py [--camera C --max-iters 1000] [--out gpurun_out/probe_steps_C.npz]"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import black_hole_ray_marching_amd as bh  # noqa: E402
from bench import CAMERAS  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--width", type=int, default=4096)
p.add_argument("--height", type=int, default=2048)
p.add_argument("--max-iters", type=int, default=512)
p.add_argument("--camera", default="A")
p.add_argument("--out", default="")
a = p.parse_args()
W, H = a.width, a.height
scene = bh.Scene(W, H, sky=bh.synthetic_sky(4096, 2048), max_iters=a.max_iters, math=bh.BH_MATH_EXACT)
if a.camera != "A":
    scene.update(bh.Camera.look_at(*CAMERAS[a.camera], W, H))
dev = torch.device("cuda")
col = torch.empty((H, W, 4), dtype=torch.float16, device=dev)
bo = torch.empty_like(col)
steps = torch.zeros((H, W), dtype=torch.int16, device=dev)
nrk = torch.zeros((H, W), dtype=torch.int16, device=dev)
fate = torch.zeros((H, W), dtype=torch.uint8, device=dev)
for _ in range(4):
    scene.render(col, bo, fmt=bh.BH_OUT_RGBA16F, dbg_n_rk=nrk, dbg_fate=fate, dbg_steps=steps)
torch.cuda.synchronize()
st = steps.cpu().numpy().astype(np.int32) & 0xFFFF
nr = nrk.cpu().numpy().astype(np.int32) & 0xFFFF
fa = fate.cpu().numpy()


def tiles(x):
    return x.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)


ts, tn = tiles(st), tiles(nr)
mx = ts.max(1)
rep = {"config": {"width": W, "height": H, "max_iters": a.max_iters, "camera": a.camera},
       "sum_executed_steps": int(st.sum()), "sum_n_rk": int(nr.sum()),
       "sum_wave_steps_executed": int(mx.sum()), "sum_wave_steps_n_rk": int(tn.max(1).sum()),
       "fates": {int(k): int(v) for k, v in zip(*np.unique(fa, return_counts=True))}}
for th in (48, 100, 200, 400, 800):
    sel = mx >= th
    rep[f"tiles_executed_ge_{th}"] = {"tiles": int(sel.sum()), "wave_steps_beyond": int((mx[sel] - th).sum()),
                                      "mean_lanes_ge": float((ts[sel] >= th).sum(1).mean()) if sel.any() else 0.0}
order = np.argsort(-mx)[:12]
rep["longest_tiles"] = [{"tile": int(t), "max_steps": int(mx[t]), "lanes_ge_half": int((ts[t] >= mx[t] // 2).sum()),
                         "n_rk_of_longest": int(tn[t][np.argmax(ts[t])]),
                         "fate_of_longest": int(tiles(fa)[t][np.argmax(ts[t])])} for t in order]
print(json.dumps(rep, indent=1))
if a.out:
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(a.out, steps=st.astype(np.uint16), n_rk=nr.astype(np.uint16), fate=fa)
