"""Seeded random frame sizes through the bloom chain (AUTO) against the oracle, one process:
    python tools/bloom_sweep.py [--n 60 --seed 1 --max-w 4200 --max-h 2300]
prints one JSON line per size that differs, then a summary line; --trace: each size before its launch (a fault then
names its size)."""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import black_hole_ray_marching_amd as bh  # noqa: E402
import oracle  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=60)
p.add_argument("--seed", type=int, default=1)
p.add_argument("--max-w", type=int, default=4200)
p.add_argument("--max-h", type=int, default=2300)
p.add_argument("--trace", action="store_true")
a = p.parse_args()
rng = np.random.default_rng(a.seed)
scene = bh.Scene(16, 16, sky=bh.synthetic_sky())
bad, forms = 0, {}
for i in range(a.n):
    W, H, L = int(rng.integers(1, a.max_w)), int(rng.integers(1, a.max_h)), int(rng.integers(1, 6))
    kinds = sorted({f for f, *_ in bh.bloom_check(W, H, L)})  # the host's dry-run check first
    if a.trace:
        print(json.dumps({"i": i, "W": W, "H": H, "levels": L, "forms": kinds}), flush=True)
    r = np.random.default_rng(W * 31 + H * 7 + L)
    col = r.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
    bo = r.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
    bo[..., :3] = np.where(r.random((H, W, 1)) < 0.05, bo[..., :3], 0)
    if i % 2 == 0:
        col[..., 3] = 255
        bo[..., 3] = 255
    c, b = torch.from_numpy(col).cuda(), torch.from_numpy(bo).cuda()
    out = torch.zeros_like(c)
    scene.bloom(c, b, out, levels=L, schedule=bh.BH_BLOOM_AUTO, width=W, height=H)
    torch.cuda.synchronize()
    got, want = out.cpu().numpy(), oracle.bloom(col, bo, L)
    for f in kinds:
        forms[f] = forms.get(f, 0) + 1
    if not np.array_equal(got, want):
        bad += 1
        d = np.argwhere(got != want)
        print(json.dumps({"W": W, "H": H, "levels": L, "differing": int(len(d)), "first": d[:4].tolist(), "forms": kinds}),
              flush=True)
    del c, b, out
print(json.dumps({"sizes": a.n, "bad": bad, "forms_seen": forms}), flush=True)
