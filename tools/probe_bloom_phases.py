"""Where a wave of the quad separable up pass (up_sepq_kernel) spends its lifetime (diagnostic; needs a
library whose bloom TU is built with -DBH_BLOOM_PHASES=1:
    tools/build_bloom_variant.sh bphase -DBH_BLOOM_PHASES=1
    BH_LIB=tools/variants/bphase.so python tools/probe_bloom_phases.py --width 1920 --height 1080)
Every wave adds the shader cycles of four phases to its kernel's slot (FP 28 / 40 / 60 tiles): the footprint,
own-texel and table loads issued and the tables staged; the tile decoded and written, up to the barrier; the
8 taps; the epilogue's stores.  Prints mean cycles per wave and each phase's share of the lifetime."""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import black_hole_ray_marching_amd as bh  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--width", type=int, default=1920)
p.add_argument("--height", type=int, default=1080)
p.add_argument("--levels", type=int, default=3)
p.add_argument("--chains", type=int, default=20)
args = p.parse_args()
W, H = args.width, args.height
lib = C.CDLL(os.environ["BH_LIB"])
lib.bh_bloom_phases_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
scene = bh.Scene(W, H, sky=bh.synthetic_sky(), max_iters=512, math=bh.BH_MATH_EXACT)
col = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
bo = torch.empty_like(col)
out = torch.empty_like(col)
scene.render(col, bo, fmt=bh.BH_OUT_BGRA8_SRGB)
for _ in range(10):
    scene.bloom(col, bo, out, levels=args.levels)
torch.cuda.synchronize()
buf = (C.c_ulonglong * 24)()
assert lib.bh_bloom_phases_read(buf, 1) == 0
for _ in range(args.chains):
    scene.bloom(col, bo, out, levels=args.levels)
torch.cuda.synchronize()
assert lib.bh_bloom_phases_read(buf, 1) == 0
names = ["loads+tables", "tile+barrier", "taps", "epilogue"]
res = {}
for k, fp in enumerate((28, 40, 60)):
    v = list(buf[8 * k:8 * k + 8])
    if v[0] == 0:
        continue
    life = v[1] / v[0]
    res[f"sepq{fp}"] = {"waves_per_chain": v[0] / args.chains, "lifetime_cycles": round(life, 1),
                        "phases_cycles": {n: round(v[2 + i] / v[0], 1) for i, n in enumerate(names)},
                        "phases_share": {n: round(v[2 + i] / v[1], 4) for i, n in enumerate(names)}}
print(json.dumps({"width": W, "height": H, "levels": args.levels, "kernels": res}))
scene.close()
