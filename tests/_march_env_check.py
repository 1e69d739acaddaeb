"""Run by tests/test_gpu_parity.py in a child process (the library reads its A/B switches once per process):
exact-math renders under the environment this process was started with -- cameras A and E (capped "Zeno"
rays), three frames each so that the temporal order is learned and then repeated -- against the oracle, bit
for bit (both targets, RGBA32F).  Exit status 0 = every frame equal."""
import sys

import numpy as np
import torch

import black_hole_ray_marching_amd as bh
import oracle
from tests._cases import camera_uniform, uniforms


def main():
    W, H, cap = 256, 128, 512
    sky = bh.synthetic_sky(512, 256)
    scene = bh.Scene(W, H, sky=sky, max_iters=cap, math=bh.BH_MATH_EXACT)
    col = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    bo = torch.zeros_like(col)
    bad = 0
    for cam in ("A", "E"):
        cu = camera_uniform(cam, W, H)
        scene.camera_uniform = cu
        want = oracle.render_rows(cu.to_bytes(), bytes(uniforms().to_c()), sky, W, H, cap, bh.BH_SCENE_DEFAULT)
        for _ in range(3):
            col.zero_()
            bo.zero_()
            scene.render(col, bo)
            torch.cuda.synchronize()
            ok = np.array_equal(col.cpu().numpy().view(np.uint32), want[0].view(np.uint32)) and \
                np.array_equal(bo.cpu().numpy().view(np.uint32), want[1].view(np.uint32))
            if not ok:
                print(cam, "differs")
                bad += 1
    scene.close()
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
