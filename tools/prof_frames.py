"""Render K frames of the headline workload (no CPU leg): a small driver for rocprofv3 runs."""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=5)
    p.add_argument("--math", choices=["fast", "exact"], default="exact")
    p.add_argument("--schedule", choices=["tile", "tile-static", "pair", "persistent"], default="tile")
    p.add_argument("--width", type=int, default=4096)
    p.add_argument("--height", type=int, default=2048)
    p.add_argument("--max-iters", type=int, default=512)
    a = p.parse_args()
    import torch
    import black_hole_ray_marching_amd as bh
    sky = bh.synthetic_sky(4096, 2048)
    sc = bh.Scene(a.width, a.height, sky=sky, max_iters=a.max_iters,
                  math=bh.BH_MATH_FAST if a.math == "fast" else bh.BH_MATH_EXACT)
    col = torch.empty((a.height, a.width, 4), dtype=torch.float16, device="cuda")
    bo = torch.empty_like(col)
    sched = {"tile": bh.BH_SCHED_TILE, "tile-static": bh.BH_SCHED_TILE | bh.BH_SCHED_FLAG_STATIC_ORDER,
             "pair": bh.BH_SCHED_PAIR, "persistent": bh.BH_SCHED_PERSISTENT}[a.schedule]
    for _ in range(a.frames):
        sc.render(col, bo, fmt=bh.BH_OUT_RGBA16F, schedule=sched)
    torch.cuda.synchronize()
    print("frames done", a.frames)


if __name__ == "__main__":
    main()
