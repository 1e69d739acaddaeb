"""Frames in flight: throughput of consecutive frames (or one rank's shards of them) so that one frame's
serial tail overlaps other frames' bulk, two ways: `streams` issues single-frame launches round-robin
on D HIP streams of one ctx (per-stream temporal order state, include/bh_render.h); `batch` renders D
frames per bh_render_frames launch on one stream.  Wall time per frame over K frames.

    python tools/probe_inflight.py [--frames 4096x2048,8192x4096] [--shards 1,8] [--depths 1,2,4,8]
                                   [--modes streams,batch]"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", default="4096x2048,8192x4096")
    p.add_argument("--shards", default="1,8")
    p.add_argument("--depths", default="1,2,4,8")
    p.add_argument("--modes", default="streams,batch")
    p.add_argument("--cap", type=int, default=512)
    p.add_argument("--k", type=int, default=96)
    p.add_argument("--variant", choices=["auto", "issue", "latency"], default="auto")
    args = p.parse_args()
    import torch
    import black_hole_ray_marching_amd as bh
    dev = torch.device("cuda:0")
    sky = bh.synthetic_sky()
    fmt = bh.BH_OUT_RGBA16F
    sched = {"auto": 0, "issue": bh.BH_SCHED_FLAG_ISSUE_ORDER, "latency": bh.BH_SCHED_FLAG_LATENCY}[args.variant]
    for fr in args.frames.split(","):
        W, H = map(int, fr.split("x"))
        scene = bh.Scene(W, H, sky=sky, max_iters=args.cap, math=bh.BH_MATH_EXACT)
        for S in map(int, args.shards.split(",")):
            for mode in args.modes.split(","):
                for D in map(int, args.depths.split(",")):
                    streams = [torch.cuda.Stream(dev) for _ in range(D if mode == "streams" else 1)]
                    if S == 1:
                        bufs = [(torch.empty((H, W, 4), dtype=torch.float16, device=dev),
                                 torch.empty((H, W, 4), dtype=torch.float16, device=dev)) for _ in range(D)]
                        kw = dict(layout=bh.BH_LAYOUT_ROWMAJOR)
                    else:
                        nt = bh.shard_tile_count(W, H, 0, S)
                        bufs = [(torch.empty((nt, bh.tile_bytes(bh.BH_LAYOUT_TILES_RGBM, fmt)), dtype=torch.uint8,
                                             device=dev), None) for _ in range(D)]
                        kw = dict(layout=bh.BH_LAYOUT_TILES_RGBM, shard_index=0, shard_count=S)

                    def run(k):
                        if mode == "streams":
                            for i in range(k):
                                c, b = bufs[i % D]
                                scene.render(c, b, fmt=fmt, stream=streams[i % D], schedule=sched, **kw)
                        else:
                            for _ in range(0, k, D):
                                scene.render_frames([c for c, _ in bufs], None if S > 1 else [b for _, b in bufs],
                                                    fmt=fmt, stream=streams[0], schedule=sched, **kw)

                    run(4 * D + 8)
                    torch.cuda.synchronize()
                    k = (args.k + D - 1) // D * D
                    t0 = time.perf_counter()
                    run(k)
                    torch.cuda.synchronize()
                    ms = (time.perf_counter() - t0) / k * 1e3
                    print(json.dumps({"frame": fr, "S": S, "mode": mode, "variant": args.variant, "depth": D, "ms_per_frame": round(ms, 4),
                                      "frame_Mpix_per_s": round(W * H / ms / 1e3, 1)}), flush=True)
        scene.close()


if __name__ == "__main__":
    main()
