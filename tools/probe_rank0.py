"""Rank 0's per-frame GPU work in bench.py's N>1 path, on one GPU: its own shard render of D frames per
launch (BH_LAYOUT_TILES_RGBM, col only; render stream) with the unpack of the previous launch's D
gathered frames into both row-major targets (bh_tiles_unpack_rgbm, side stream, throttled to
`rows` tile rows in flight) running beside it.  Every other rank only renders, so
max(rank 0's frame, a shard render) is the predicted N-GPU frame time without the transport.

    python tools/probe_rank0.py [--n 2,4,8] [--frame 4096x2048] [--D 8] [--rows 16] [--it 12]
Prints one JSON line per N: render alone, render + unpack, unpack alone (ms per frame)."""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", default="2,4,8")
    p.add_argument("--frame", default="4096x2048")
    p.add_argument("--D", type=int, default=8)
    p.add_argument("--rows", default="16", help="comma list of tile rows in flight (0 = all)")
    p.add_argument("--it", type=int, default=12)
    a = p.parse_args()
    import torch
    import black_hole_ray_marching_amd as bh
    from black_hole_ray_marching_amd import multigpu
    dev = torch.device("cuda:0")
    W, H = (int(v) for v in a.frame.split("x"))
    fmt = bh.BH_OUT_RGBA16F
    D = a.D
    sky = bh.synthetic_sky(4096, 2048)
    for n, rows in ((int(v), int(r)) for v in a.n.split(",") for r in a.rows.split(",")):
        stride = multigpu.packed_stride(W, H, n)
        tb = bh.tile_bytes(bh.BH_LAYOUT_TILES_RGBM, fmt)
        scene = bh.Scene(W, H, sky=sky, device=0, max_iters=512, math=bh.BH_MATH_EXACT)
        mine = torch.empty((D * stride, tb), dtype=torch.uint8, device=dev)
        # the gathered launch: every rank's block of D frames (rank 0's own block is rendered for real
        # once, the others are copies of it: the unpack's cost does not depend on the pixel values)
        scene.render_frames([mine[f * stride:(f + 1) * stride] for f in range(D)], None, fmt=fmt,
                            layout=bh.BH_LAYOUT_TILES_RGBM, shard_index=0, shard_count=n)
        gathered = mine.repeat(n, 1)
        cols = [torch.empty((H, W, 4), dtype=torch.float16, device=dev) for _ in range(D)]
        bos = [torch.empty_like(c) for c in cols]
        rs = torch.cuda.current_stream()
        ss = torch.cuda.Stream()

        def render():
            scene.render_frames([mine[f * stride:(f + 1) * stride] for f in range(D)], None, fmt=fmt,
                                layout=bh.BH_LAYOUT_TILES_RGBM, shard_index=0, shard_count=n, stream=rs)

        def unpack():
            for f in range(D):
                bh.tiles_unpack_rgbm(gathered[f * stride:], cols[f], bos[f], W, H, n, D * stride, fmt,
                                     stream=ss, rows_in_flight=rows)

        def run(k, do_render, do_unpack):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(k):
                if do_render:
                    render()
                if do_unpack:
                    ev = torch.cuda.Event()
                    ev.record(rs)
                    ss.wait_event(ev)          # the bench's side stream waits for the receive
                    unpack()                   # renders never wait for it (double-buffered receive)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / (k * D) * 1e3

        for _ in range(3):
            run(4, True, True)
        out = {"n": n, "frame": f"{W}x{H}", "frames_per_launch": D, "unpack_rows_in_flight": rows,
               "shard_tiles": bh.shard_tile_count(W, H, 0, n),
               "render_ms": round(run(a.it, True, False), 4),
               "render_plus_unpack_ms": round(run(a.it, True, True), 4),
               "unpack_only_ms": round(run(a.it, False, True), 4)}
        print(json.dumps(out), flush=True)
        scene.close()


if __name__ == "__main__":
    main()
