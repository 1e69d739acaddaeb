"""Predicted strong-scaling curve without an 8-GPU node (VERDICT r01 "Next round" 3a): the fixed
4096x2048 (north_star) and 8192x4096 (BASELINE config 4) frames cut into S = 1, 2, 4, 8 shards
((tx + 3*ty) % S tiles), each shard rendered ALONE on this GPU as a rank renders it (RGBM, col only),
HIP events around each launch.  The slowest shard bounds the N=S frame (gather and unpack overlap the
next frame); its longest executed ray chain is the serial floor.

    python tools/probe_shard.py [--frames 4096x2048,8192x4096] [--shards 1,2,4,8] [--cap 512] [--it 20]
Prints one JSON line per (frame, S)."""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", default="4096x2048,8192x4096")
    p.add_argument("--shards", default="1,2,4,8")
    p.add_argument("--cap", type=int, default=512)
    p.add_argument("--camera", default="A")
    p.add_argument("--it", type=int, default=20)
    p.add_argument("--variant", choices=["auto", "issue", "latency"], default="auto")
    args = p.parse_args()
    import torch
    import black_hole_ray_marching_amd as bh
    from black_hole_ray_marching_amd import multigpu
    dev = torch.device("cuda:0")
    sky = bh.synthetic_sky(4096, 2048)
    cams = {"B": ((0.0, 3.0, -20.0), (0.0, 0.0, 0.0)), "C": ((0.0, 6.0, -12.0), (0.0, 0.0, 0.0))}
    sched = bh.BH_SCHED_TILE | {"auto": 0, "issue": bh.BH_SCHED_FLAG_ISSUE_ORDER,
                                "latency": bh.BH_SCHED_FLAG_LATENCY}[args.variant]
    fmt = bh.BH_OUT_RGBA16F

    def timed(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.it)]
        for a, b in ev:
            a.record(); fn(); b.record()
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))

    base = {}
    for fr in args.frames.split(","):
        W, H = map(int, fr.split("x"))
        scene = bh.Scene(W, H, sky=sky, device=0, max_iters=args.cap, math=bh.BH_MATH_EXACT)
        if args.camera != "A":
            scene.update(bh.Camera.look_at(*cams[args.camera], W, H))
        for S in map(int, args.shards.split(",")):
            per = []
            for k in range(S):
                if S == 1:
                    col = torch.empty((H, W, 4), dtype=torch.float16, device=dev)
                    bo = torch.empty_like(col)
                    kw = dict(layout=bh.BH_LAYOUT_ROWMAJOR)
                    shape = (H, W)
                else:
                    nt = bh.shard_tile_count(W, H, k, S)
                    col = torch.empty((nt, bh.tile_bytes(bh.BH_LAYOUT_TILES_RGBM, fmt)), dtype=torch.uint8, device=dev)
                    bo = None
                    kw = dict(layout=bh.BH_LAYOUT_TILES_RGBM, shard_index=k, shard_count=S)
                    shape = (nt * 64,)
                ms = timed(lambda: scene.render(col, bo, fmt=fmt, schedule=sched, **kw))
                steps = torch.zeros(shape, dtype=torch.int16, device=dev)
                scene.render(col, bo, fmt=fmt, schedule=sched, dbg_steps=steps, **kw)
                torch.cuda.synchronize()
                s = steps.cpu().numpy().view(np.uint16).astype(np.int64)
                per.append((ms, int(s.sum()), int(s.max())))
            ms = [x[0] for x in per]
            worst = max(ms)
            if S == 1:
                base[fr] = worst
            print(json.dumps({"frame": fr, "cap": args.cap, "camera": args.camera, "S": S,
                              "max_shard_ms": round(worst, 4), "mean_shard_ms": round(float(np.mean(ms)), 4),
                              "min_shard_ms": round(min(ms), 4),
                              "predicted_speedup": round(base.get(fr, worst) / worst, 3),
                              "predicted_efficiency": round(base.get(fr, worst) / worst / S, 3),
                              "sum_steps_per_shard": [x[1] for x in per],
                              "longest_chain_steps": max(x[2] for x in per)}), flush=True)
        scene.close()


if __name__ == "__main__":
    main()
