"""Predicted multi-GPU line of the driver's protocol (`bench.py --gpus N --steps K --warmup W`) from one-GPU
probes plus the xGMI link model.  Reads tools/probe_rank0.py's JSON lines (rank 0's render +
unpack, another rank's render, the unpack alone; ms per frame) and prints, per (N, frames per launch D,
transport, rank-0 ratio), the steady-state frame time and the line's ms per frame including the drain.

Model (one step = one batch of D frames, batch i's gather overlaps batch i+1's render):
  render    = max(rank 0's render + unpack (side stream), another rank's render)        [probe]
  ingress   = (1 - s0) * frame_bytes / (links * link_GBps)   rank 0 receives N - 1 shards over N - 1 links
  steady    = max(render, ingress)
  drain     = (ingress + unpack) / K per frame: the last batch's gather and unpack follow its render
  predicted = steady + drain;  speedup = one_gpu_ms / predicted
s0 = rank 0's tile share (its tiles cross no link); frame_bytes = tiles * tile_bytes.  link_GBps: one xGMI
link's rate in one direction (MI355X: 7 links of 153.6 GB/s bidirectional, 76.8 per direction; RCCL's
achieved share of it is the model's unknown, `--link-eff`).

    python tools/scale_model.py probe.jsonl --one-gpu-ms 0.556 [--k 20] [--link-gbps 76.8] [--link-eff 1.0]
--rebalance: per (N, D, transport) also the best rank-0 share on the grid unit 20 (weights [w0, 20, ...]):
rank 0's and another rank's render scale with their tile counts (per-tile rates from the probe row),
rank 0 adds the unpack, and the ingress shrinks with rank 0's share."""
import argparse
import json


def frontier(one_gpu_ms: float, k: int, n: int = 8, tiles: int = 131072, unpack_ms: float = 0.0365):
    """What N = 8 needs for a given speedup, from the model alone: for each link rate, shard per-tile cost and
    transport size, the best rank-0 share s0 (fine grid) and the predicted ms per frame (drain included).
    Rank 0 renders s0 of the tiles and unpacks every frame (unpack_ms, not overlapped: DESIGN.md §7); the
    others render (1 - s0) / (n - 1) each; rank 0 receives (1 - s0) of the frame over n - 1 links."""
    print(f"frontier: N = {n}, {tiles} tiles, rank-0 unpack {unpack_ms} ms/frame, K = {k}; 7x needs "
          f"<= {one_gpu_ms / 7:.4f} ms/frame")
    print("| link GB/s per direction | shard ns/tile | transport B/px | best s0 | render | ingress | predicted | vs 1 GPU |")
    print("|---|---|---|---|---|---|---|---|")
    for link in (76.8, 153.6, float("inf")):
        for ns in (4.36, 4.20, 4.07):
            for bpp in (5.375, 4.8, 4.3):
                best = None
                for i in range(0, 401):
                    s0 = i / 2000.0
                    r0 = ns * 1e-6 * tiles * s0 + unpack_ms
                    r1 = ns * 1e-6 * tiles * (1.0 - s0) / (n - 1)
                    ing = 0.0 if link == float("inf") else (1.0 - s0) * tiles * 64 * bpp / ((n - 1) * link * 1e9) * 1e3
                    st = max(r0, r1, ing)
                    pr = st + (ing + unpack_ms) / k
                    if best is None or pr < best[0]:
                        best = (pr, s0, max(r0, r1), ing)
                pr, s0, rr, ing = best
                print(f"| {link} | {ns} | {bpp} | {s0:.3f} | {rr:.4f} | {ing:.4f} | {pr:.4f} | {one_gpu_ms / pr:.2f}x |")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("probe", nargs="?", default="")
    p.add_argument("--frontier", action="store_true", help="print the model's requirement table (no probe file)")
    p.add_argument("--one-gpu-ms", type=float, required=True)
    p.add_argument("--k", type=int, default=20)
    p.add_argument("--link-gbps", type=float, default=76.8)
    p.add_argument("--link-eff", type=float, default=1.0)
    p.add_argument("--rebalance", action="store_true")
    p.add_argument("--unpack-ms", type=float, default=0.0365,
                   help="frontier: rank 0's exposed unpack per frame (0: fully hidden under its render)")
    a = p.parse_args()
    if a.frontier:
        frontier(a.one_gpu_ms, a.k, unpack_ms=a.unpack_ms)
        return
    rows = [json.loads(x) for x in open(a.probe) if x.startswith("{")]
    print(f"one GPU {a.one_gpu_ms} ms/frame, K = {a.k}, link {a.link_gbps} GB/s x {a.link_eff} per direction")
    print("| N | D | transport | weights | render (ms) | ingress (ms) | binds | predicted ms/frame | Gpix/s | vs 1 GPU |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        n = r["n"]
        if n < 2:  # a one-GPU reference row (probe --n 1): nothing crosses a link
            continue
        W, H = (int(v) for v in r["frame"].split("x"))
        tiles = ((W + 7) // 8) * ((H + 7) // 8)
        w = r.get("weights") or [1] * n
        s0 = w[0] / sum(w)
        frame_bytes = tiles * r["tile_bytes"]
        ingress = (1.0 - s0) * frame_bytes / ((n - 1) * a.link_gbps * a.link_eff * 1e9) * 1e3
        render = max(r["rank0_render_plus_unpack_ms"], r["rank1_render_ms"])
        steady = max(render, ingress)
        pred = steady + (ingress + r["unpack_only_ms"]) / a.k
        print(f"| {n} | {r['frames_per_launch']} | {r.get('transport', 'rgbm')} | {w if r.get('weights') else 'even'} | "
              f"{render:.4f} | {ingress:.4f} | {'render' if render >= ingress else 'xGMI'} | {pred:.4f} | "
              f"{W * H / pred / 1e6:.1f} | {a.one_gpu_ms / pred:.2f}x |")
        if a.rebalance and r.get("tiles"):
            t0, t1 = r["tiles"]
            a0 = r["rank0_render_ms"] / t0
            a1 = r["rank1_render_ms"] / t1
            U = r["rank0_render_plus_unpack_ms"] - r["rank0_render_ms"]
            best = None
            for w0 in range(0, 41):
                tot = w0 + 20 * (n - 1)
                s0n = w0 / tot
                r0 = a0 * tiles * s0n + U
                r1 = a1 * tiles * 20 / tot
                ing = (1.0 - s0n) * frame_bytes / ((n - 1) * a.link_gbps * a.link_eff * 1e9) * 1e3
                st = max(r0, r1, ing)
                pr = st + (ing + r["unpack_only_ms"]) / a.k
                if best is None or pr < best[0]:
                    best = (pr, w0, r0, r1, ing)
            pr, w0, r0, r1, ing = best
            bind = "rank 0" if r0 >= max(r1, ing) else ("render" if r1 >= ing else "xGMI")
            print(f"| {n} | {r['frames_per_launch']} | {r.get('transport', 'rgbm')} | rebalanced [{w0}, 20, ...] | "
                  f"{max(r0, r1):.4f} | {ing:.4f} | {bind} | {pr:.4f} | {W * H / pr / 1e6:.1f} | {a.one_gpu_ms / pr:.2f}x |")


if __name__ == "__main__":
    main()
