"""Per-frame kernel time of the first K frames after Scene creation (VERDICT r01 "Next round" 6):
separates the temporal cost order's learning (frame 1 runs the centre-out order) from the clock
ramp.  Series (one frame per launch unless named _D8, HIP events):
  learned             the learned order, cold start (first Scene of the process)
  static              the static centre-out order (no learning)
  learned_after_idle  the learned order again after a 1 s idle gap
  hot_learned         a NEW Scene (fresh order state: frame 1 centre-out, then learning) started
                      right after 300 frames of another Scene kept the GPU busy: if this series
                      starts at its steady time on frame 2, the cold series' slow descent is the
                      clock, not the order
  hot_static          the static order, right after hot_learned
  idle_D8             1 s idle, then a NEW Scene at 8 frames per launch (the bench's default), per-frame
                      time of each launch

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
    cols = [torch.empty_like(col) for _ in range(8)]
    bos = [torch.empty_like(col) for _ in range(8)]
    out = {}

    def series(flag, frames, D=1):
        scene = bh.Scene(4096, 2048, sky=sky, max_iters=512, math=bh.BH_MATH_EXACT)
        n = max(1, frames // D)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for s, e in ev:
            s.record()
            if D == 1:
                scene.render(col, bo, fmt=bh.BH_OUT_RGBA16F, schedule=bh.BH_SCHED_TILE | flag)
            else:
                scene.render_frames(cols[:D], bos[:D], fmt=bh.BH_OUT_RGBA16F, schedule=bh.BH_SCHED_TILE | flag)
            e.record()
        torch.cuda.synchronize()
        scene.close()
        return [round(s.elapsed_time(e) / D, 4) for s, e in ev]

    out["learned"] = series(0, a.frames)
    out["static"] = series(bh.BH_SCHED_FLAG_STATIC_ORDER, a.frames)
    time.sleep(1.0)
    out["learned_after_idle"] = series(0, a.frames)
    series(0, 300)  # keep the GPU busy (untimed use of the result)
    out["hot_learned"] = series(0, a.frames)
    out["hot_static"] = series(bh.BH_SCHED_FLAG_STATIC_ORDER, a.frames)
    time.sleep(1.0)
    out["idle_D8"] = series(0, 8 * 12, D=8)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
