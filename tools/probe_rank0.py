"""Rank 0's per-frame GPU work in bench.py's N>1 path, on one GPU: its own shard render of D frames per
launch (BH_LAYOUT_TILES_RGBM, col only; render stream) with the unpack of the previous launch's D
gathered frames into both row-major targets (side stream, `rows` tile rows in flight) running beside
it, and another rank's shard render alone.  max(rank 0's frame, another rank's) is the predicted
N-GPU frame time without the transport.  --root-ratio: rank 0's share relative to the others'
(weighted partition, bh_partition; 1 = the plain interleave).

    python tools/probe_rank0.py [--n 2,4,8] [--frame 4096x2048] [--D 8] [--rows 64] [--root-ratio 1,auto]
Prints one JSON line per (N, rows, ratio), ms per frame."""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def masked_streams(torch, k):
    """(render stream on every CU but k, unpack stream on those k: every (n_cu / k)-th mask bit), as torch streams"""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    hip.hipExtStreamCreateWithCUMask.argtypes = [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(C.c_uint32)]
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (n_cu + 31) // 32
    side = {i * (n_cu // k) for i in range(k)}
    out = []
    for bits in ([c for c in range(n_cu) if c not in side], sorted(side)):
        m = (C.c_uint32 * words)()
        for b in bits:
            m[b // 32] |= 1 << (b % 32)
        h = C.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(C.byref(h), words, m) == 0
        out.append(torch.cuda.ExternalStream(h.value))
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", default="2,4,8")
    p.add_argument("--frame", default="4096x2048")
    p.add_argument("--D", type=int, default=8)
    p.add_argument("--rows", default="64", help="comma list of tile rows in flight (0 = all)")
    p.add_argument("--root-ratio", default="1", help="comma list: numbers or 'auto'")
    p.add_argument("--it", type=int, default=12)
    p.add_argument("--transport", choices=["rgbm", "rgbm14"], default="rgbm14")
    p.add_argument("--side-priority", default="0", help="comma list: the unpack stream's priority (0 normal, -1 high)")
    p.add_argument("--render-streams", type=int, default=1, help="launches alternate over this many streams")
    p.add_argument("--tag", default="", help="copied into every line (e.g. the A/B variant)")
    p.add_argument("--cu-split", default="0", help="comma list: k > 0 runs the unpack on k CUs and the render on the "
                                                   "others (hipExtStreamCreateWithCUMask), 0 = shared CUs")
    a = p.parse_args()
    import torch
    import black_hole_ray_marching_amd as bh
    from black_hole_ray_marching_amd import multigpu
    dev = torch.device("cuda:0")
    W, H = (int(v) for v in a.frame.split("x"))
    fmt = bh.BH_OUT_RGBA16F
    D = a.D
    sky = bh.synthetic_sky(4096, 2048)
    layout = bh.BH_LAYOUT_TILES_RGBM14 if a.transport == "rgbm14" else bh.BH_LAYOUT_TILES_RGBM
    ufmt = fmt | bh.BH_UNPACK_RGBM14 if a.transport == "rgbm14" else fmt
    tb = bh.tile_bytes(layout, fmt)
    for n in (int(v) for v in a.n.split(",")):
        for rr in a.root_ratio.split(","):
            ratio = multigpu.auto_root_ratio(n) if rr == "auto" else float(rr)
            weights = multigpu.root_weights(n, ratio)
            part = bh.Partition(W, H, weights) if len(set(weights)) > 1 else None
            counts = part.counts if part else [bh.shard_tile_count(W, H, k, n) for k in range(n)]
            stride = max(counts)
            kw = dict(layout=layout, shard_count=n, **({"partition": part} if part else {}))
            for rows, sp, cus in ((int(r), int(q), int(c)) for r in a.rows.split(",") for q in a.side_priority.split(",")
                                  for c in a.cu_split.split(",")):
                scene = bh.Scene(W, H, sky=sky, device=0, max_iters=512, math=bh.BH_MATH_EXACT)
                bufs = [torch.empty((D * stride, tb), dtype=torch.uint8, device=dev) for _ in range(2)]
                K1 = 1 if n > 1 else 0  # n = 1: the whole frame in the packed layout (rank 1 := rank 0)
                for k in sorted({0, K1}):  # the gathered launch: rank 0's and rank 1's blocks rendered for real
                    scene.render_frames([bufs[k][f * stride:f * stride + counts[k]] for f in range(D)], None, fmt=fmt,
                                        shard_index=k, **kw)
                gathered = torch.cat([bufs[0], bufs[1]] + [bufs[1]] * (n - 2), 0) if n > 1 else bufs[0]
                cols = [torch.empty((H, W, 4), dtype=torch.float16, device=dev) for _ in range(D)]
                bos = [torch.empty_like(c) for c in cols]
                rs = torch.cuda.current_stream()
                ss = torch.cuda.Stream(priority=sp)
                rss = [rs] + [torch.cuda.Stream() for _ in range(a.render_streams - 1)]
                if cus:
                    rs, ss = masked_streams(torch, cus)
                    rss = [rs]
                nl = [0]

                def render(k):
                    # with several render streams consecutive launches alternate, so that one launch's last
                    # waves overlap the next launch's first (each stream has its own learned order)
                    st = rss[nl[0] % len(rss)]
                    nl[0] += 1
                    scene.render_frames([bufs[k][f * stride:f * stride + counts[k]] for f in range(D)], None, fmt=fmt,
                                        shard_index=k, stream=st, **kw)
                    return st

                def unpack():
                    for f in range(D):
                        if part:
                            bh.tiles_unpack_rgbm_partition(gathered[f * stride:], cols[f], bos[f], part, D * stride,
                                                           ufmt, stream=ss, rows_in_flight=rows)
                        else:
                            bh.tiles_unpack_rgbm(gathered[f * stride:], cols[f], bos[f], W, H, n, D * stride, ufmt,
                                                 stream=ss, rows_in_flight=rows)

                def run(k, shard, do_render, do_unpack):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(k):
                        st = render(shard) if do_render else rs
                        if do_unpack:
                            ev = torch.cuda.Event()
                            ev.record(st)
                            ss.wait_event(ev)  # the bench's side stream waits for the receive
                            unpack()           # renders never wait for it (double-buffered receive)
                    torch.cuda.synchronize()
                    return (time.perf_counter() - t0) / (k * D) * 1e3

                for _ in range(3):
                    run(4, 0, True, True)
                    run(2, K1, True, False)
                r0 = run(a.it, 0, True, True)
                r1 = run(a.it, K1, True, False)
                out = {"tag": a.tag, "n": n, "frame": f"{W}x{H}", "frames_per_launch": D, "unpack_rows_in_flight": rows,
                       "transport": a.transport, "tile_bytes": tb, "side_priority": sp, "render_streams": a.render_streams,
                       "unpack_cus": cus or None,
                       "root_ratio": round(ratio, 4), "weights": weights if part else None, "tiles": (counts + counts)[:2],
                       "rank0_render_ms": round(run(a.it, 0, True, False), 4), "rank0_render_plus_unpack_ms": round(r0, 4),
                       "rank1_render_ms": round(r1, 4), "unpack_only_ms": round(run(a.it, 0, False, True), 4),
                       "predicted_frame_ms": round(max(r0, r1), 4)}
                out["rank1_ns_per_tile"] = round(r1 * 1e6 / counts[K1], 4)
                print(json.dumps(out), flush=True)
                scene.close()
            if part:
                part.close()


if __name__ == "__main__":
    main()
