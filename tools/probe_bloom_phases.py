"""Where a wave of the quad separable up pass (up_sepq_kernel) and of the fix-up pass (fixup_gather_kernel)
spends its lifetime, and how the launch's waves overlap in time (diagnostic; needs a library whose bloom TU is built with -DBH_BLOOM_PHASES=1:
    tools/build_bloom_variant.sh bphase -DBH_BLOOM_PHASES=1
    BH_LIB=tools/variants/bphase.so python tools/probe_bloom_phases.py --width 1920 --height 1080)
Every wave writes one record (bh_bloom.hip, BH_BLOOM_PHASES; plain stores, no shared counter): its global
start and end (s_memrealtime, 100 MHz) and the shader cycles of four phases -- footprint, own-texel and table
loads issued and the tables staged; the tile decoded and written, up to the barrier; the 8 taps; the epilogue's
stores.  Per launch: the span first start -> last end, the mean wave lifetime and phase shares, the ramp (first
start -> the moment the most waves are resident), the tail (last wave start -> last end) and the mean number
of resident waves over the span."""
import argparse
import ctypes as C
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import black_hole_ray_marching_amd as bh  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--width", type=int, default=1920)
p.add_argument("--height", type=int, default=1080)
p.add_argument("--levels", type=int, default=3)
p.add_argument("--chains", type=int, default=5)
args = p.parse_args()
W, H = args.width, args.height
lib = C.CDLL(os.environ["BH_LIB"])
lib.bh_bloom_phases_read.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_int]
lib.bh_bloom_phases_geometry.restype = C.c_uint32
geo = lib.bh_bloom_phases_geometry()
SLOTS, MAXW = geo >> 24, geo & 0xFFFFFF
scene = bh.Scene(W, H, sky=bh.synthetic_sky(), max_iters=512, math=bh.BH_MATH_EXACT)
col = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
bo = torch.empty_like(col)
out = torch.empty_like(col)
scene.render(col, bo, fmt=bh.BH_OUT_BGRA8_SRGB)
for _ in range(10):
    scene.bloom(col, bo, out, levels=args.levels)
torch.cuda.synchronize()
hdr = np.zeros((SLOTS, 4), np.uint32)
rec = np.zeros((SLOTS, MAXW, 8), np.uint32)
P32 = C.POINTER(C.c_uint32)
lib.bh_bloom_phases_read(hdr.ctypes.data_as(P32), None, 1)
names = ["loads+tables", "tile+barrier", "taps", "epilogue"]
acc = defaultdict(lambda: defaultdict(list))
for _ in range(args.chains):
    scene.bloom(col, bo, out, levels=args.levels)
    n = lib.bh_bloom_phases_read(hdr.ctypes.data_as(P32), rec.ctypes.data_as(P32), 1)
    assert 0 < n <= SLOTS, n
    for k in range(n):
        fp, epi, blocks, ow = (int(x) for x in hdr[k])
        nw = min(blocks * 4, MAXW)
        r = rec[k, :nw].astype(np.int64)
        r = r[(r[:, 0] != 0) | (r[:, 1] != 0)]  # waves with no record (a fix-up's dead tail lanes)
        t0 = r[:, 0] - r[:, 0].min()
        t1 = r[:, 1] - r[:, 0].min()
        span = t1.max()  # 10 ns ticks
        grid = np.linspace(0, span, 200)
        resident = np.array([np.count_nonzero((t0 <= g) & (t1 > g)) for g in grid])
        key = f"sepq{fp}/{epi} {ow}" if fp else f"fixup/{epi} {ow}"
        a = acc[key]
        a["fixup"] = [fp == 0]
        a["span_us"].append(span / 100.0)
        a["wave_us"].append(float((t1 - t0).mean()) / 100.0)
        a["ramp_us"].append(float(grid[int(resident.argmax())]) / 100.0)
        a["tail_us"].append(float(span - t0.max()) / 100.0)
        a["mean_resident"].append(float(resident.mean()))
        a["peak_resident"].append(float(resident.max()))
        a["waves"].append(len(r))
        for i, nm in enumerate(names):
            a[nm].append(float(r[:, 2 + i].mean()))
        a["life_cycles"].append(float(r[:, 6].mean()))
res = {}
# the fix-up's phases (fixup_gather_kernel): list and plan entries in registers; tables staged; texel words
# arrived; the pixel computed and stored
fix_names = ["entries", "tables", "texels", "compute+store"]
for key, a in acc.items():
    life = np.mean(a["life_cycles"])
    nm_out = fix_names if a["fixup"][0] else names
    res[key] = {k: round(float(np.mean(a[k])), 2) for k in ("span_us", "wave_us", "ramp_us", "tail_us", "mean_resident",
                                                           "peak_resident", "waves")}
    res[key]["life_cycles"] = round(float(life), 1)
    res[key]["phases_cycles"] = {o: round(float(np.mean(a[nm])), 1) for o, nm in zip(nm_out, names)}
    res[key]["phases_share"] = {o: round(float(np.mean(a[nm]) / life), 4) for o, nm in zip(nm_out, names)}
print(json.dumps({"width": W, "height": H, "levels": args.levels, "chains": args.chains, "launches": res}))
scene.close()
