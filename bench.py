#!/usr/bin/env python3
"""Headline benchmark: Mpix/s of the geodesic ray-march at 4096x2048, 512 RK-step cap
(BASELINE.json configs[2]), plus max |delta pixel| against the CPU oracle (the WGSL restatement).

A "step" is one full frame: one pass of the hot path (`Scene::render` -> the HIP march kernel)
over the synthetic 4096x2048 frame, sky already resident in HBM.  N=1: one GPU renders the whole
frame.  N>1 (torch.distributed, one process per GPU, RCCL): weak scaling — the frame grows with
N (about 8.4 Mpix per GPU, aspect 2:1, e.g. 8192x4096 at N=4), every rank renders its
(tx + 3*ty) % N share of 8x8 tiles, the tile-packed `col` shares are gathered to rank 0 over RCCL
and unpacked there; the timed step includes the gather and the unpack.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Mpix/s at 4096×2048, 512 RK steps; max |Δpixel| vs WGSL ref"
F_STEP = 209          # flop-equivalents per completed RK step, surfaces on
F_STEP_NO_SURF = 159
PEAK_FP32_TFLOPS = 157.3   # MI355X FP32 vector peak (MI355X_MICROARCH.md, chip table)
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--math", choices=["fast", "exact"], default="fast")
    p.add_argument("--fmt", choices=["rgba16f", "rgba32f"], default="rgba16f")
    p.add_argument("--width", type=int, default=0)
    p.add_argument("--height", type=int, default=0)
    p.add_argument("--max-iters", type=int, default=512)
    p.add_argument("--camera", choices=["A", "B", "C"], default="A")
    p.add_argument("--schedule", choices=["persistent", "tile"], default="persistent")
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline / parity leg")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = all cores in this process's affinity")
    return p.parse_args()


def frame_size(n: int, args) -> tuple[int, int]:
    if args.width and args.height:
        return args.width, args.height
    if n == 1:
        return 4096, 2048
    w = int(round(4096 * math.sqrt(n) / 8.0)) * 8
    return w, w // 2


def main() -> None:
    args = parse()
    import torch
    import torch.distributed as dist

    import black_hole_ray_marching_amd as bh

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    n = max(world, 1)
    torch.cuda.set_device(local)
    if n > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    W, H = frame_size(n, args)
    cap = args.max_iters
    fmt = bh.BH_OUT_RGBA16F if args.fmt == "rgba16f" else bh.BH_OUT_RGBA32F
    ch_dtype = torch.float16 if fmt == bh.BH_OUT_RGBA16F else torch.float32
    bpp = bh.BYTES_PER_PIXEL[fmt]
    math_mode = bh.BH_MATH_FAST if args.math == "fast" else bh.BH_MATH_EXACT

    sky = bh.synthetic_sky(4096, 2048)
    scene = bh.Scene(W, H, sky=sky, device=local, max_iters=cap, math=math_mode)
    if args.camera != "A":
        spec = {"B": ((0.0, 3.0, -20.0), (0.0, 0.0, 0.0)), "C": ((0.0, 6.0, -12.0), (0.0, 0.0, 0.0))}[args.camera]
        scene.update(bh.Camera.look_at(spec[0], spec[1], W, H))
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream(dev)
    sched = bh.BH_SCHED_PERSISTENT if args.schedule == "persistent" else bh.BH_SCHED_TILE
    _render = scene.render

    def render(*a, **kw):
        return _render(*a, schedule=sched, **kw)
    scene.render = render

    if n == 1:
        col = torch.empty((H, W, 4), dtype=ch_dtype, device=dev)
        bo = torch.empty((H, W, 4), dtype=ch_dtype, device=dev)

        def step():
            scene.render(col, bo, fmt=fmt, stream=stream)
        px_per_step = W * H
        my_tiles = None
    else:
        counts = [bh.shard_tile_count(W, H, k, n) for k in range(n)]
        stride = max(counts)
        my_tiles = counts[rank]
        col = torch.empty((stride * 64, 4), dtype=ch_dtype, device=dev)
        bo = torch.empty((stride * 64, 4), dtype=ch_dtype, device=dev)
        gathered = [torch.empty_like(col) for _ in range(n)] if rank == 0 else None
        frame = torch.empty((H, W, 4), dtype=ch_dtype, device=dev) if rank == 0 else None
        packed_all = torch.empty((n * stride * 64, 4), dtype=ch_dtype, device=dev) if rank == 0 else None

        def step():
            scene.render(col, bo, fmt=fmt, stream=stream, layout=bh.BH_LAYOUT_TILES, shard_index=rank,
                         shard_count=n)
            dist.gather(col, gathered if rank == 0 else None, dst=0)
            if rank == 0:
                torch.cat(gathered, out=packed_all)
                bh.tiles_unpack(packed_all, frame, W, H, n, stride, bpp, stream=stream)
        px_per_step = W * H  # whole-job pixels per step (all ranks)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    # timed region: barrier + synchronize on both sides; per-launch HIP events on the render stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if n > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        if n == 1:
            step()
            ev[i][1].record(stream)
        else:
            scene.render(col, bo, fmt=fmt, stream=stream, layout=bh.BH_LAYOUT_TILES, shard_index=rank,
                         shard_count=n)
            ev[i][1].record(stream)
            dist.gather(col, gathered if rank == 0 else None, dst=0)
            if rank == 0:
                torch.cat(gathered, out=packed_all)
                bh.tiles_unpack(packed_all, frame, W, H, n, stride, bpp, stream=stream)
    torch.cuda.synchronize(dev)
    if n > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if n > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    kern_avg_s = float(np.mean(kern_ms)) / 1e3

    # algorithmic work of one launch: sum of completed RK steps over this rank's pixels (deterministic)
    nrk_buf = torch.zeros(col.shape[:-1], dtype=torch.int16, device=dev)
    if n == 1:
        scene.render(col, bo, fmt=fmt, stream=stream, dbg_n_rk=nrk_buf)
    else:
        scene.render(col, bo, fmt=fmt, stream=stream, layout=bh.BH_LAYOUT_TILES, shard_index=rank,
                     shard_count=n, dbg_n_rk=nrk_buf)
    torch.cuda.synchronize(dev)
    nrk = nrk_buf.cpu().numpy().view(np.uint16)
    if my_tiles is not None:
        nrk = nrk[: my_tiles * 64]
    sum_nrk = int(nrk.astype(np.int64).sum())
    my_px = W * H if n == 1 else int(min(my_tiles * 64, W * H))

    if rank != 0:
        if n > 1:
            dist.destroy_process_group()
        return

    value = px_per_step * args.steps / elapsed / 1e6
    flops = sum_nrk * F_STEP
    achieved_tf = flops / kern_avg_s / 1e12
    out_bytes = my_px * bpp * 2
    sky_bytes = sky.nbytes
    achieved_gbs = (out_bytes + sky_bytes) / kern_avg_s / 1e9
    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mpix/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (splitmix64-seeded 4096x2048 RGBA8 sRGB sky; reference default camera)",
        "config": {
            "workload": f"{W}x{H} frame, cap {cap} RK steps, disc+markers+sky, camera {args.camera}, "
                        f"{args.fmt} col+blackout" + ("" if n == 1 else ", 8x8 tiles (tx+3ty)%N + RCCL gather of col"),
            "width": W, "height": H, "max_iters": cap, "camera": args.camera, "math": args.math,
            "format": args.fmt, "parallelism": "single GPU" if n == 1 else f"tile-sharded x{n}",
        },
        "kernel": {"name": f"march_kernel ({args.math})", "avg_ms": round(kern_avg_s * 1e3, 5),
                   "min_ms": round(float(np.min(kern_ms)), 5), "sum_n_rk": sum_nrk,
                   "mean_n_rk": round(sum_nrk / my_px, 4), "fps_kernel": round(1.0 / kern_avg_s, 2)},
        "roofline": {"bound": "valu", "achieved": round(achieved_tf, 3), "peak": PEAK_FP32_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved_tf / PEAK_FP32_TFLOPS, 5),
                     "traffic": _pmc_traffic(W, H, cap, args),
                     "note": f"{F_STEP} flop-eq per completed RK step x sum(n_rk) / avg launch time; "
                             "FP32 VALU-bound (no MFMA-shaped work)"},
        "roofline_hbm": {"bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / PEAK_HBM_GBS, 5),
                         "note": "algorithmic bytes: col+blackout outputs + sky texture once"},
    }
    if not args.no_cpu:
        result["cpu_baseline"], result["parity"] = _cpu_leg(scene, sky, W, H, cap, args, col, bo, fmt, stream, n)
    else:
        result["cpu_baseline"] = None
    print(json.dumps(result))
    if n > 1:
        dist.destroy_process_group()


def _pmc_traffic(W, H, cap, args):
    """HBM bytes per launch from committed rocprofv3 PMC passes (profiles/pmc_traffic.json), or None."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        key = f"{W}x{H}_cap{cap}_{args.math}_{args.fmt}"
        e = d.get(key)
        return None if e is None else e.get("hbm_bytes_per_launch")
    except Exception:
        return None


def _cpu_leg(scene, sky, W, H, cap, args, col, bo, fmt, stream, n):
    """cpu_baseline (oracle, host cores, bounded sample) + parity of the GPU frame on that sample."""
    import torch

    import black_hole_ray_marching_amd as bh
    import oracle

    # the GPU box's CPU share is 16 cores (os.cpu_count() shows the whole machine there)
    threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
    # bounded sample: every 8th row of the same frame (1/8 of the pixels, all image regions)
    step8 = 8
    rows = list(range(3, H, step8))
    cu, U = scene.camera_uniform.to_bytes(), bytes(scene.uniforms.to_c())
    oracle.render_rows(cu, U, sky, W, H, cap, 3, 0, 64, threads=threads, row_step=step8)  # warm
    t0 = time.perf_counter()
    o_col, _, o_nrk, o_fate = oracle.render_rows(cu, U, sky, W, H, cap, 3, 3, H, threads=threads, row_step=step8)
    cpu_s = time.perf_counter() - t0
    cpu_px = len(rows) * W
    cpu_baseline = {"value": round(cpu_px / cpu_s / 1e6, 4), "unit": "Mpix/s", "cores": threads, "kind": "port",
                    "sample": f"{len(rows)} rows (every {step8}th) x {W} px of the same {W}x{H} cap-{cap} frame, "
                              f"C oracle -O2 -ffp-contract=off, OpenMP {threads} threads, {cpu_s:.2f} s"}
    parity = None
    if n == 1:
        # fp32 output of the same (fast) kernel for a precise delta
        c32 = torch.empty((H, W, 4), dtype=torch.float32, device=col.device)
        nrk = torch.empty((H, W), dtype=torch.int16, device=col.device)
        fate = torch.empty((H, W), dtype=torch.uint8, device=col.device)
        scene.render(c32, None, fmt=bh.BH_OUT_RGBA32F, stream=stream, dbg_n_rk=nrk, dbg_fate=fate)
        torch.cuda.synchronize()
        gc = c32[rows].cpu().numpy()
        gn = nrk[rows].cpu().numpy().view(np.uint16)
        gf = fate[rows].cpu().numpy()
        oc, on, of = o_col, o_nrk, o_fate
        match = (gf == of) & (gn == on)
        d = np.abs(gc[..., :3] - oc[..., :3]).max(axis=-1)
        parity = {"vs": "oracle/bh_oracle.c (normative restatement of src/black_hole_maybe.wgsl)",
                  "sample_px": int(match.size), "fate_nrk_match": round(float(match.mean()), 6),
                  "max_abs_delta_matched": float(d[match].max()), "max_abs_delta_all": float(d.max()),
                  "tolerance": 1e-4, "math": args.math}
    return cpu_baseline, parity


if __name__ == "__main__":
    main()
