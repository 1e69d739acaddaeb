"""Per-rank march time at the N-GPU weak-scaling frame (one shard rendered on this GPU) vs the
N=1 frame: shows the per-wave cost of the shard tile mapping.  python tools/probe_shard.py"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import torch
    import black_hole_ray_marching_amd as bh
    from black_hole_ray_marching_amd import multigpu
    dev = torch.device("cuda:0")
    sky = bh.synthetic_sky(4096, 2048)

    def t(fn, it=30):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(it)]
        for a, b in ev:
            a.record(); fn(); b.record()
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in ev) / it

    for n in (1, 2, 4, 8):
        W, H = multigpu.weak_scaling_frame(n)
        scene = bh.Scene(W, H, sky=sky, device=0, max_iters=512, math=bh.BH_MATH_EXACT)
        for k in ([0] if n == 1 else [0, n - 1]):
            if n == 1:
                col = torch.empty((H, W, 4), dtype=torch.float16, device=dev); bo = torch.empty_like(col)
                kw = dict(layout=bh.BH_LAYOUT_ROWMAJOR)
                px = W * H
            else:
                nt = bh.shard_tile_count(W, H, k, n)
                col = torch.empty((nt, 3, 64), dtype=torch.float16, device=dev); bo = torch.empty_like(col)
                kw = dict(layout=bh.BH_LAYOUT_TILES_RGB, shard_index=k, shard_count=n)
                px = nt * 64
            ms = t(lambda: scene.render(col, bo, fmt=bh.BH_OUT_RGBA16F, **kw))
            print(json.dumps({"n": n, "shard": k, "frame": f"{W}x{H}", "px": px, "ms": round(ms, 4),
                              "Mpix_per_s": round(px / ms / 1e3, 1)}))
        scene.close()


if __name__ == "__main__":
    main()
