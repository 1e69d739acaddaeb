"""Why an orbiting camera path renders slower than the fixed camera A (bench.py --camera-path orbit):
for camera A rotated about the y axis by a few angles, one frame's capped rays (fate CAP), the ones
that ran every step (no cycle fast-forward), the tiles holding them, and the per-frame kernel time of
that camera repeated (a perfectly predicted temporal order), 1 and 8 frames per launch.

    python tools/orbit_probe.py [--angles 0,0.2,1,5]"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--angles", default="0,0.2,1,5")
    a = p.parse_args()
    import torch
    import black_hole_ray_marching_amd as bh
    import bench
    W, H, cap = 4096, 2048, 512
    sky = bh.synthetic_sky()
    scene = bh.Scene(W, H, sky=sky, max_iters=cap, math=bh.BH_MATH_EXACT)
    cols = [torch.empty((H, W, 4), dtype=torch.float16, device="cuda") for _ in range(8)]
    bos = [torch.empty_like(c) for c in cols]
    nrk = torch.zeros((H, W), dtype=torch.int16, device="cuda")
    steps = torch.zeros((H, W), dtype=torch.int16, device="cuda")
    fate = torch.zeros((H, W), dtype=torch.uint8, device="cuda")
    for ang in (float(v) for v in a.angles.split(",")):
        cu = bench.orbit_camera(bh, "A", 0, W, H) if ang == 0 else None
        if cu is None:
            bench.ORBIT_DEG_PER_FRAME = ang
            cu = bench.orbit_camera(bh, "A", 1, W, H)
        scene.camera_uniform = cu
        scene.render(cols[0], bos[0], fmt=bh.BH_OUT_RGBA16F, dbg_n_rk=nrk, dbg_fate=fate, dbg_steps=steps)
        torch.cuda.synchronize()
        f, s = fate.cpu().numpy(), steps.cpu().numpy().view(np.uint16)
        capped = f == bh.BH_FATE_CAP if hasattr(bh, "BH_FATE_CAP") else f == 3
        full = capped & (s >= cap)
        ty, tx = np.nonzero(full)
        tiles = len(set(zip((ty // 8).tolist(), (tx // 8).tolist())))
        res = {"angle_deg": ang, "capped": int(capped.sum()), "capped_full_chain": int(full.sum()),
               "tiles_with_full_chain": tiles, "sum_steps": int(s.astype(np.int64).sum())}
        for D in (1, 8):
            for _ in range(60 // D + 2):
                scene.render_frames(cols[:D], bos[:D], fmt=bh.BH_OUT_RGBA16F)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(max(2, 96 // D))]
            for e0, e1 in ev:
                e0.record()
                scene.render_frames(cols[:D], bos[:D], fmt=bh.BH_OUT_RGBA16F)
                e1.record()
            torch.cuda.synchronize()
            res[f"ms_per_frame_D{D}"] = round(float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev])) / D, 4)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
