"""Run by tests/test_gpu_bloom.py in a child process (the library reads its A/B switches once per process):
the fused chain under the environment this process was started with, against oracle/bh_bloom_oracle.c,
bit-exact, on the frames given as HxW[:alpha] arguments.  Exit status 0 = every frame equal."""
import sys

import numpy as np
import torch

import black_hole_ray_marching_amd as bh
import oracle


def main(args):
    scene = bh.Scene(16, 16, sky=bh.synthetic_sky())
    bad = 0
    for a in args:
        shape, _, alpha = a.partition(":")
        H, W = (int(v) for v in shape.split("x"))
        rng = np.random.default_rng(W * 11 + H)
        col = rng.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
        bo = rng.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
        bo[..., :3] = np.where(rng.random((H, W, 1)) < 0.05, bo[..., :3], 0)
        if alpha != "any":
            col[..., 3] = 255
            bo[..., 3] = 255
        c, b = torch.from_numpy(col).cuda(), torch.from_numpy(bo).cuda()
        out = torch.zeros_like(c)
        scene.bloom(c, b, out, levels=3, schedule=bh.BH_BLOOM_AUTO, width=W, height=H)
        torch.cuda.synchronize()
        got, want = out.cpu().numpy(), oracle.bloom(col, bo, 3)
        if not np.array_equal(got, want):
            print(a, "differs at", np.argwhere(got != want)[:5].tolist())
            bad += 1
    scene.close()
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
