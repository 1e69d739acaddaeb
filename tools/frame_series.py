"""Per-frame kernel time of the first K frames after Scene creation (VERDICT r01 "Next round" 6):
separates the temporal cost order's learning (frame 1 runs the centre-out order) from the clock
ramp.  Three series: the learned order, the static centre-out order (no learning: what is left is the
clock), and the learned order again after a 1 s idle gap.  One frame per launch, HIP events.

    python tools/frame_series.py [--frames 50]"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=50)
    a = p.parse_args()
    import torch
    import black_hole_ray_marching_amd as bh
    sky = bh.synthetic_sky()
    col = torch.empty((2048, 4096, 4), dtype=torch.float16, device="cuda")
    bo = torch.empty_like(col)
    out = {}
    for name, flag in (("learned", 0), ("static", bh.BH_SCHED_FLAG_STATIC_ORDER), ("learned_after_idle", 0)):
        if name == "learned_after_idle":
            time.sleep(1.0)
        scene = bh.Scene(4096, 2048, sky=sky, max_iters=512, math=bh.BH_MATH_EXACT)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.frames)]
        for s, e in ev:
            s.record()
            scene.render(col, bo, fmt=bh.BH_OUT_RGBA16F, schedule=bh.BH_SCHED_TILE | flag)
            e.record()
        torch.cuda.synchronize()
        out[name] = [round(s.elapsed_time(e), 4) for s, e in ev]
        scene.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
