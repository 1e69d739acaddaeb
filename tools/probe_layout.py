"""The headline frame (4096x2048, cap 512, exact, RGBA16F col + blackout) rendered into each output
layout: row-major vs tile-packed stores.  python tools/probe_layout.py"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import torch
    import black_hole_ray_marching_amd as bh
    dev = torch.device("cuda:0")
    W, H = 4096, 2048
    scene = bh.Scene(W, H, sky=bh.synthetic_sky(4096, 2048), device=0, max_iters=512, math=bh.BH_MATH_EXACT)

    def t(fn, it=50):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(it)]
        for a, b in ev:
            a.record(); fn(); b.record()
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in ev) / it

    nt = bh.shard_tile_count(W, H, 0, 1)
    for rep in range(2):
        for name, layout, shape in (("rowmajor", bh.BH_LAYOUT_ROWMAJOR, (H, W, 4)),
                                    ("tiles", bh.BH_LAYOUT_TILES, (nt * 64, 4)),
                                    ("tiles_rgb", bh.BH_LAYOUT_TILES_RGB, (nt, 3, 64))):
            col = torch.empty(shape, dtype=torch.float16, device=dev); bo = torch.empty_like(col)
            for target in ("col+bo", "col"):
                b = bo if target == "col+bo" else None
                ms = t(lambda: scene.render(col, b, fmt=bh.BH_OUT_RGBA16F, layout=layout))
                print(json.dumps({"layout": name, "targets": target, "ms": round(ms, 4)}))


if __name__ == "__main__":
    main()
