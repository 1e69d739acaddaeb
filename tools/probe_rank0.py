"""Rank 0's per-frame GPU work at the N-GPU weak-scaling frame, on one GPU: its own shard render
(render stream) with the unpack of the previous gathered frame (side stream) running beside it.
Prints the frame time alone and with the unpack overlapped.  python tools/probe_rank0.py [N]"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import torch
    import black_hole_ray_marching_amd as bh
    from black_hole_ray_marching_amd import multigpu
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda:0")
    W, H = multigpu.weak_scaling_frame(n)
    stride = multigpu.packed_stride(W, H, n)
    scene = bh.Scene(W, H, sky=bh.synthetic_sky(4096, 2048), device=0, max_iters=512, math=bh.BH_MATH_EXACT)
    nt = bh.shard_tile_count(W, H, 0, n)
    col = torch.empty((stride, 3, 64), dtype=torch.float16, device=dev)
    bo = torch.empty_like(col)
    gathered = torch.zeros((n * stride, 3, 64), dtype=torch.float16, device=dev)
    frame = torch.empty((H, W, 4), dtype=torch.float16, device=dev)
    # BH_RENDER_PRIO=1: the render stream at high priority (the unpack stream stays at the default)
    import os
    hi = os.environ.get("BH_RENDER_PRIO") == "1"
    rs = torch.cuda.Stream(priority=-1) if hi else torch.cuda.current_stream()
    ss = torch.cuda.Stream()
    # BH_UNPACK_ROWS=k: the unpack's tile rows in flight (bh_tiles_unpack_rgb_rows; 0 = all)
    rows = int(os.environ.get("BH_UNPACK_ROWS", "0"))
    # BH_VARIANT=issue|latency: force a build of the exact kernels (default: bh_render's choice)
    sched = {"": 0, "issue": bh.BH_SCHED_FLAG_ISSUE_ORDER, "latency": bh.BH_SCHED_FLAG_LATENCY}[os.environ.get("BH_VARIANT", "")]

    def render():
        scene.render(col, bo, fmt=bh.BH_OUT_RGBA16F, layout=bh.BH_LAYOUT_TILES_RGB, shard_index=0, shard_count=n,
                     stream=rs, schedule=sched)

    def unpack():
        bh.tiles_unpack_rgb(gathered, frame, W, H, n, stride, bh.BH_OUT_RGBA16F, stream=ss, rows_in_flight=rows)

    def run(k, with_unpack, unpack_only=False):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            if not unpack_only:
                render()
            if with_unpack:
                unpack()
                ev = torch.cuda.Event(); ev.record(ss); rs.wait_event(ev)  # next frame waits (pipeline depth 1)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    for _ in range(2):
        run(5, True)
    out = {"n": n, "frame": f"{W}x{H}", "tiles": nt, "render_prio_high": hi, "variant": os.environ.get("BH_VARIANT", "auto"), "unpack_rows_in_flight": rows,
           "render_ms": round(run(50, False), 4), "render_plus_unpack_ms": round(run(50, True), 4),
           "unpack_only_ms": round(run(50, True, True), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
