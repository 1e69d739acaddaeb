"""The serial floor of the frame's tail (VERDICT r01 "Next round" 3c): one 8x8 tile of capped,
non-cycling rays marched ALONE on the GPU, at several caps; the slope of kernel time over the
executed chain length is a lone wave's time per RK step.

The tile is taken from the 4096x2048 camera-A frame: the tile with the most rays that run to the cap
without entering a cycle.  A 8x8 frame whose camera corners are the affine restriction of the big
frame's corners to that tile (same barycentric interpolation, rescaled) marches almost the same
rays (not bit-identical: the interpolation rounds differently; the chain lengths are reported).

    python tools/probe_chain.py [--caps 512,1024,2048,4096] [--variant issue|latency|both]"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--caps", default="512,1024,2048,4096")
    p.add_argument("--variant", default="both")
    p.add_argument("--tiles", type=int, default=3)
    p.add_argument("--it", type=int, default=10)
    args = p.parse_args()
    import torch
    import black_hole_ray_marching_amd as bh
    sky = bh.synthetic_sky()
    W, H, cap0 = 4096, 2048, 512
    big = bh.Scene(W, H, sky=sky, max_iters=cap0, math=bh.BH_MATH_EXACT)
    col = torch.empty((H, W, 4), device="cuda")
    steps = torch.zeros((H, W), dtype=torch.int16, device="cuda")
    nrk = torch.zeros((H, W), dtype=torch.int16, device="cuda")
    big.render(col, None, dbg_steps=steps, dbg_n_rk=nrk)
    torch.cuda.synchronize()
    s = steps.cpu().numpy().view(np.uint16).astype(np.int64)
    n = nrk.cpu().numpy().view(np.uint16).astype(np.int64)
    long_ = ((s == cap0) & (n == cap0)).reshape(H // 8, 8, W // 8, 8).sum(axis=(1, 3))
    order = np.argsort(-long_.ravel())[:args.tiles]
    C = big.camera_uniform.world_tri.astype(np.float64)  # rows C0, C1, C2
    variants = {"issue": bh.BH_SCHED_FLAG_ISSUE_ORDER, "latency": bh.BH_SCHED_FLAG_LATENCY}
    if args.variant != "both":
        variants = {args.variant: variants[args.variant]}
    for ti in order:
        ty, tx = divmod(int(ti), W // 8)
        # l0_big = tx/1024 + l0'/512, l2_big = ty/512 + l2'/256 for the 8x8 frame's barycentrics l0', l2'
        C1 = C[1] + (tx * 8 / (2 * W)) * (C[0] - C[1]) + (ty * 8 / (2 * H)) * (C[2] - C[1])
        C0 = C1 + (C[0] - C[1]) * (16 / (2 * W))
        C2 = C1 + (C[2] - C[1]) * (16 / (2 * H))
        small = bh.Scene(8, 8, sky=sky, max_iters=cap0, math=bh.BH_MATH_EXACT)
        for i, c in enumerate((C0, C1, C2)):
            for k in range(3):
                small.camera_uniform.c.world_tri[i][k] = float(np.float32(c[k]))
        out = torch.empty((8, 8, 4), device="cuda")
        st = torch.zeros((8, 8), dtype=torch.int16, device="cuda")
        for vname, vflag in variants.items():
            rows = []
            for cap in map(int, args.caps.split(",")):
                small.max_iters = cap
                sched = bh.BH_SCHED_TILE | vflag
                for _ in range(3):
                    small.render(out, None, schedule=sched)
                torch.cuda.synchronize()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.it)]
                for a, b in ev:
                    a.record(); small.render(out, None, schedule=sched); b.record()
                torch.cuda.synchronize()
                ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
                small.render(out, None, schedule=sched, dbg_steps=st)
                torch.cuda.synchronize()
                chain = int(st.cpu().numpy().view(np.uint16).max())
                rows.append((cap, ms, chain))
            (c0, m0, ch0), (c1, m1, ch1) = rows[0], rows[-1]
            slope = (m1 - m0) / (ch1 - ch0) * 1e3 if ch1 != ch0 else None
            print(json.dumps({"tile": [tx, ty], "capped_noncycling_rays": int(long_.ravel()[ti]), "variant": vname,
                              "runs": [{"cap": c, "ms": round(m, 4), "chain_steps": ch} for c, m, ch in rows],
                              "us_per_step_alone": None if slope is None else round(slope, 4)}), flush=True)
        small.close()
    big.close()


if __name__ == "__main__":
    main()
