"""One frame of the bloom chain (AUTO) against the oracle, for bisecting a mismatch over the library's run-time
switches: the parent runs the frame once per switch set given, each in a child process (the library reads its
switches once per process), with test_gpu_bloom's inputs (test_bloom_bitexact_random_sizes).
    python tools/bloom_bisect.py H W LEVELS [ENV=1[,ENV2=1] | default ...]
Arms run in the order given (no arm: the default only); the first child that fails (a GPU fault, an exception)
ends the run with its exit status -- nothing more runs on the GPU after a fault."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def child(H, W, L):
    import numpy as np
    import torch
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    import black_hole_ray_marching_amd as bh
    import oracle
    from test_gpu_bloom import _img
    rng = np.random.default_rng(W * 31 + H * 7 + L)
    col, bo = _img(rng, H, W), _img(rng, H, W, sparse=True)
    scene = bh.Scene(16, 16, sky=bh.synthetic_sky())
    c, b = torch.from_numpy(col).cuda(), torch.from_numpy(bo).cuda()
    out = torch.zeros_like(c)
    scene.bloom(c, b, out, levels=L, schedule=bh.BH_BLOOM_AUTO, width=W, height=H)
    torch.cuda.synchronize()
    got, want = out.cpu().numpy(), oracle.bloom(col, bo, L)
    d = np.argwhere(got != want)
    px = np.unique(d[:, :2], axis=0) if len(d) else d
    print(json.dumps({"env": os.environ.get("BISECT_TAG", ""), "differing_pixels": int(len(px)),
                      "rows": [int(px[:, 0].min()), int(px[:, 0].max())] if len(px) else None,
                      "cols": [int(px[:, 1].min()), int(px[:, 1].max())] if len(px) else None,
                      "first": px[:6].tolist(),
                      "launches": [x[0] for x in bh.bloom_check(W, H, L)]}), flush=True)


if __name__ == "__main__":
    if os.environ.get("BISECT_CHILD"):
        child(*(int(v) for v in sys.argv[1:4]))
        sys.exit(0)
    H, W, L = sys.argv[1:4]
    for arm in sys.argv[4:] or ["default"]:
        arm = "" if arm == "default" else arm
        env = dict(os.environ, BISECT_CHILD="1", BISECT_TAG=arm or "default", PYTHONPATH=str(ROOT))
        for kv in filter(None, arm.split(",")):
            k, v = kv.split("=")
            env[k] = v
        print(json.dumps({"arm": arm or "default", "W": int(W), "H": int(H), "levels": int(L)}), flush=True)
        r = subprocess.run([sys.executable, __file__, H, W, L], env=env, capture_output=True, text=True, timeout=300)
        print(r.stdout.strip() or r.stderr[-1500:], flush=True)
        if r.returncode != 0:
            print(r.stderr[-1500:], flush=True)
            sys.exit(r.returncode)
