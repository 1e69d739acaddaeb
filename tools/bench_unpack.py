"""Rank 0's unpack of the gathered shards (bh_tiles_unpack_rgb / bh_tiles_unpack) at the bench's
weak-scaling frame sizes: average kernel time (HIP events) and algorithmic GB/s (packed bytes read +
frame bytes written).  One JSON line per (N, layout).

    python tools/bench_unpack.py [--iters 50]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    import torch

    import black_hole_ray_marching_amd as bh
    from black_hole_ray_marching_amd import multigpu

    p = argparse.ArgumentParser()
    p.add_argument("--iters", type=int, default=50)
    args = p.parse_args()
    dev = torch.device("cuda:0")
    for n in (2, 4, 8):
        W, H = multigpu.weak_scaling_frame(n)
        stride = multigpu.packed_stride(W, H, n)
        frame = torch.empty((H, W, 4), dtype=torch.float16, device=dev)
        for layout in ("tiles_rgb", "tiles"):
            shape = (n * stride, 3, 64) if layout == "tiles_rgb" else (n * stride * 64, 4)
            packed = torch.randn(shape, dtype=torch.float32, device=dev).to(torch.float16)

            def run():
                if layout == "tiles_rgb":
                    bh.tiles_unpack_rgb(packed, frame, W, H, n, stride, bh.BH_OUT_RGBA16F)
                else:
                    bh.tiles_unpack(packed, frame, W, H, n, stride, 8)

            for _ in range(3):
                run()
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
            for a, b in ev:
                a.record()
                run()
                b.record()
            torch.cuda.synchronize()
            ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
            nbytes = packed.numel() * 2 + frame.numel() * 2
            print(json.dumps({"n": n, "frame": f"{W}x{H}", "layout": layout, "avg_ms": round(ms, 5),
                              "algorithmic_bytes": nbytes, "GB_per_s": round(nbytes / ms / 1e6, 1)}))


if __name__ == "__main__":
    main()
