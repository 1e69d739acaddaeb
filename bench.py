#!/usr/bin/env python3
"""Headline benchmark: Mpix/s of the geodesic ray-march at 4096x2048 with a 512 RK-step cap
(BASELINE.json configs[2]) and the max |delta pixel| against the CPU oracle (the normative WGSL
restatement, oracle/bh_oracle.c).

A "step" is one frame: one pass of the hot path (Scene::render -> the HIP march kernel) over the
synthetic 4096x2048 frame, the sky already resident in HBM.  Default arithmetic: BH_MATH_EXACT, the
bit-exact path (the only one that can meet |delta| < 1e-4, DESIGN.md "Math modes"); RGBA16F col +
blackout targets as north_star asks.

N=1: one GPU renders the whole frame.  N>1 (torch.distributed, one process per GPU, RCCL): weak
scaling, the frame grows with N (~8.4 Mpix per GPU, aspect 2:1: 8192x4096 at N=4), each rank renders
its (tx + 3*ty) % N share of 8x8 tiles, the tile-packed `col` shares (RGB planes: alpha is always 1
and not shipped) are gathered to rank 0 in one collective and unpacked there; each timed step includes render, gather and unpack.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Mpix/s at 4096×2048, 512 RK steps; max |Δpixel| vs WGSL ref"
F_STEP = {3: 209, 0: 159}  # flop-equivalents per completed RK step (surfaces on / off), SURVEY §8d
PEAK_FP32_TFLOPS = 157.3   # MI355X FP32 vector peak (MI355X_MICROARCH.md chip table)
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec


# tile rows in flight of rank 0's unpack (bh_tiles_unpack_rgb_rows)
UNPACK_ROWS_IN_FLIGHT = 16

def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)   # SURVEY §8d timing protocol: 100 timed frames
    # SURVEY §8d asks for 10 warm-up frames; 300 (0.25 s) let the clocks settle: +1 % measured
    p.add_argument("--warmup", type=int, default=300)
    p.add_argument("--math", choices=["exact", "fast"], default="exact")
    p.add_argument("--schedule", choices=["tile", "tile-static", "pair", "persistent"], default="tile")
    p.add_argument("--variant", choices=["auto", "issue", "latency"], default="auto",
                   help="exact math: build of the march kernels (auto: per frame, include/bh_render.h)")
    p.add_argument("--fmt", choices=["rgba16f", "rgba32f", "bgra8"], default="rgba16f")
    p.add_argument("--width", type=int, default=0)
    p.add_argument("--height", type=int, default=0)
    p.add_argument("--max-iters", type=int, default=512)
    p.add_argument("--camera", choices=["A", "B", "C"], default="A")
    p.add_argument("--surfaces", choices=["on", "off"], default="on",
                   help="off = scene_flags 0 (no disc, no markers: BASELINE config 1's scene)")
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline / parity leg")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cores in this process's affinity)")
    p.add_argument("--cpu-reps", type=int, default=3)
    p.add_argument("--graph", action="store_true",
                   help="N=1: capture one frame's bh_render (order kernels + march) in a HIP graph and replay it")
    p.add_argument("--verify-gather", action="store_true",
                   help="N>1: rank 0 compares the assembled frame with its own full-frame render (bitwise)")
    return p.parse_args()


CAMERAS = {"B": ((0.0, 3.0, -20.0), (0.0, 0.0, 0.0)), "C": ((0.0, 6.0, -12.0), (0.0, 0.0, 0.0))}


def main() -> None:
    args = parse()
    import torch
    import torch.distributed as dist

    import black_hole_ray_marching_amd as bh
    from black_hole_ray_marching_amd import multigpu

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    n = max(world, 1)
    # BH_BENCH_REHEARSAL=1 (development only, never set by the driver): all ranks share cuda:0 and
    # the gloo backend, to exercise the N>1 path (sharding, pipelined gather, unpack) on a 1-GPU box
    rehearsal = os.environ.get("BH_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if n > 1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    W, H = (args.width, args.height) if args.width and args.height else multigpu.weak_scaling_frame(n)
    cap = args.max_iters
    fmt = {"rgba16f": bh.BH_OUT_RGBA16F, "rgba32f": bh.BH_OUT_RGBA32F, "bgra8": bh.BH_OUT_BGRA8_SRGB}[args.fmt]
    ch_dtype = {bh.BH_OUT_RGBA16F: torch.float16, bh.BH_OUT_RGBA32F: torch.float32,
                bh.BH_OUT_BGRA8_SRGB: torch.uint8}[fmt]
    bpp = bh.BYTES_PER_PIXEL[fmt]
    math_mode = bh.BH_MATH_EXACT if args.math == "exact" else bh.BH_MATH_FAST
    sched = {"tile": bh.BH_SCHED_TILE, "tile-static": bh.BH_SCHED_TILE | bh.BH_SCHED_FLAG_STATIC_ORDER,
             "pair": bh.BH_SCHED_PAIR, "persistent": bh.BH_SCHED_PERSISTENT}[args.schedule]
    sched |= {"auto": 0, "issue": bh.BH_SCHED_FLAG_ISSUE_ORDER, "latency": bh.BH_SCHED_FLAG_LATENCY}[args.variant]

    sky = bh.synthetic_sky(4096, 2048)
    flags = bh.BH_SCENE_DEFAULT if args.surfaces == "on" else 0
    scene = bh.Scene(W, H, sky=sky, device=local, max_iters=cap, math=math_mode, scene_flags=flags)
    if args.camera != "A":
        scene.update(bh.Camera.look_at(*CAMERAS[args.camera], W, H))
    stream = torch.cuda.current_stream(dev)

    if n == 1:
        col = torch.empty((H, W, 4), dtype=ch_dtype, device=dev)
        bo = torch.empty((H, W, 4), dtype=ch_dtype, device=dev)
        shard = dict(layout=bh.BH_LAYOUT_ROWMAJOR)
        my_px = W * H
        pipe = None
    else:
        # weak scaling: each rank renders its (tx + 3ty) % n tiles into a packed buffer; frame i's
        # gather to rank 0 (col only: rank 0 can recompute blackout_col) overlaps frame i+1's render.
        # The shards are BH_LAYOUT_TILES_RGB (alpha, always 1, is not shipped: 3/4 of the bytes into
        # rank 0's xGMI links); rank 0's unpack restores it.
        stride = multigpu.packed_stride(W, H, n)
        my_px = bh.shard_tile_count(W, H, rank, n) * 64
        bo = torch.empty((stride, 3, 64), dtype=ch_dtype, device=dev)
        frame = torch.empty((H, W, 4), dtype=ch_dtype, device=dev) if rank == 0 else None
        shard = dict(layout=bh.BH_LAYOUT_TILES_RGB, shard_index=rank, shard_count=n)

        def on_frame(i, gathered):  # issued on the pipeline's side stream (current stream here)
            # throttled: overlaps the next render on this GPU (0.78 -> 0.73 ms rank-0 frame at N=8)
            bh.tiles_unpack_rgb(gathered, frame, W, H, n, stride, fmt, stream=torch.cuda.current_stream(dev),
                                rows_in_flight=UNPACK_ROWS_IN_FLIGHT)

        pipe = multigpu.GatherPipeline(lambda: torch.empty((stride, 3, 64), dtype=ch_dtype, device=dev),
                                       rank, n, on_frame, side_stream=torch.cuda.Stream(dev))
        col = pipe.buffer(0)

    frame_no = [0]

    def render_direct(**kw):
        scene.render(col if pipe is None else pipe.buffer(frame_no[0]), bo, fmt=fmt, stream=stream,
                     schedule=sched, **shard, **kw)

    graph = None
    if args.graph and n == 1:
        render_direct()  # allocate the per-geometry buffers before capture
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            scene.render(col, bo, fmt=fmt, stream=torch.cuda.current_stream(dev), schedule=sched, **shard)

    def render(**kw):
        if graph is not None and not kw:
            graph.replay()
        else:
            render_direct(**kw)

    def exchange():
        if pipe is not None:
            pipe.submit(frame_no[0])
        frame_no[0] += 1

    for _ in range(args.warmup):
        render()
        exchange()
    if pipe is not None:
        pipe.drain()
    torch.cuda.synchronize(dev)

    # timed region: barrier + synchronize on both sides; HIP events around every render launch on
    # the stream the kernel runs on (kernel duration for the roofline)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if n > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        render()
        ev[i][1].record(stream)
        exchange()
    if pipe is not None:
        pipe.drain()
    torch.cuda.synchronize(dev)
    if n > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if n > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = np.array([a.elapsed_time(b) for a, b in ev])
    kern_avg_s = float(kern_ms.mean()) / 1e3

    gather_ok = None
    if args.verify_gather and n > 1 and rank == 0:
        ref = torch.empty((H, W, 4), dtype=ch_dtype, device=dev)
        scene.render(ref, None, fmt=fmt, stream=stream, schedule=sched)
        torch.cuda.synchronize(dev)
        gather_ok = bool(torch.equal(ref.view(torch.uint8), frame.view(torch.uint8)))
        del ref

    # algorithmic work of one launch: RK steps over this rank's pixels (deterministic).  sum_n_rk is
    # the loop's own count (what the reference iterates); sum_steps the updates actually executed
    # (lower by the cycle fast-forward of the tile schedule) -- the roofline uses the latter.
    px_shape = (H, W) if n == 1 else (stride * 64,)  # the layout's pixel index space
    nrk_buf = torch.zeros(px_shape, dtype=torch.int16, device=dev)
    steps_buf = torch.zeros(px_shape, dtype=torch.int16, device=dev)
    render(dbg_n_rk=nrk_buf, dbg_steps=steps_buf)
    torch.cuda.synchronize(dev)
    sum_nrk = int(nrk_buf.cpu().numpy().view(np.uint16).astype(np.int64).sum())
    sum_steps = int(steps_buf.cpu().numpy().view(np.uint16).astype(np.int64).sum())

    if rank == 0:
        pmc = _pmc_entry(W, H, cap, args)
        value = W * H * args.steps / elapsed / 1e6
        achieved_tf = sum_steps * F_STEP[flags] / kern_avg_s / 1e12
        alg_bytes = my_px * (bpp if n == 1 else bpp * 3 // 4) * 2 + sky.nbytes
        achieved_gbs = alg_bytes / kern_avg_s / 1e9
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
                "workload": f"{W}x{H} frame, cap {cap} RK steps, "
                            f"{'disc+markers+sky' if flags else 'sky only (no surfaces)'}, camera {args.camera}, "
                            f"{args.fmt} col+blackout, {args.math} math"
                            + ("" if n == 1 else f", 8x8 tiles (tx+3ty)%{n}, RCCL gather of col (RGB planes) to rank 0 "
                                                  "overlapped with the next frame, unpack on rank 0"),
                "width": W, "height": H, "max_iters": cap, "camera": args.camera, "math": args.math,
                "schedule": args.schedule, "format": args.fmt,
                "parallelism": ("single GPU" + (", HIP graph replay" if graph is not None else "")) if n == 1
                               else f"tile-sharded x{n}"
                               + (" (REHEARSAL: all ranks on cuda:0, gloo; not a measurement)" if rehearsal else ""),
            },
            "kernel": {"name": f"bh::{args.math}::march_{args.schedule.split('-')[0]}_kernel<{fmt}u"
                               + (", 3u>" if args.schedule.startswith("tile") and flags == 3
                                  else (", 4294967295u>" if args.schedule.startswith("tile") else ">")), "launches": args.steps,
                       "avg_ms": round(kern_avg_s * 1e3, 5), "min_ms": round(float(kern_ms.min()), 5),
                       "max_ms": round(float(kern_ms.max()), 5), "sum_n_rk": sum_nrk, "sum_steps": sum_steps,
                       "mean_n_rk": round(sum_nrk / my_px, 4), "frames_per_s": round(1.0 / kern_avg_s, 2)},
            "roofline": {"bound": "valu", "achieved": round(achieved_tf, 3), "peak": PEAK_FP32_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved_tf / PEAK_FP32_TFLOPS, 5),
                         "traffic": pmc.get("hbm_bytes_per_launch"),
                         "valu_busy": pmc.get("valu_busy_est"),
                         "valu_lane_utilization": pmc.get("valu_lane_utilization"),
                         "note": f"{F_STEP[flags]} flop-eq per executed RK step (SURVEY §8d) x sum_steps / avg "
                                 "launch time (HIP events on the render stream); FP32 VALU-bound, no "
                                 "MFMA-shaped work; traffic = HBM bytes/launch and valu_busy = VALU issue "
                                 "cycles / SIMD cycles, both from rocprofv3 PMC passes of this configuration "
                                 "(profiles/pmc_traffic.json)"},
            "roofline_hbm": {"bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": PEAK_HBM_GBS,
                             "unit": "GB/s", "frac": round(achieved_gbs / PEAK_HBM_GBS, 5),
                             "algorithmic_bytes_per_launch": alg_bytes,
                             "note": "col+blackout outputs + the sky texture read once"},
        }
        if args.no_cpu or n > 1:
            result["cpu_baseline"] = None
        else:
            result["cpu_baseline"], result["parity"] = _cpu_leg(scene, sky, W, H, cap, args, dev, stream, sched)
        if gather_ok is not None:
            result["gather_verified_bit_exact"] = gather_ok
        print(json.dumps(result))
    if n > 1:
        dist.barrier()
        dist.destroy_process_group()


def _pmc_entry(W, H, cap, args):
    """This configuration's entry of profiles/pmc_traffic.json (rocprofv3 PMC passes), or {}."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    try:
        return json.loads(p.read_text()).get(f"{W}x{H}_cap{cap}_{args.math}_{args.schedule}_{args.fmt}") or {}
    except (OSError, ValueError):
        return {}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_leg(scene, sky, W, H, cap, args, dev, stream, sched):
    """cpu_baseline: the C oracle on the host cores over the same full frame, `cpu_reps` times
    (bounded: ~1 s wall, ~15 core-seconds on the GPU box); parity: the GPU frame (fp32 output of the
    same kernel and math mode) against that oracle frame, every pixel."""
    import torch

    import black_hole_ray_marching_amd as bh
    import oracle

    threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
    cu, U = scene.camera_uniform.to_bytes(), bytes(scene.uniforms.to_c())
    oracle.render_rows(cu, U, sky, W, H, cap, scene.scene_flags, 0, 64, threads=threads)  # warm-up
    times = []
    for _ in range(max(1, args.cpu_reps)):
        t0 = time.perf_counter()
        o_col, _, o_nrk, o_fate = oracle.render_rows(cu, U, sky, W, H, cap, scene.scene_flags, threads=threads)
        times.append(time.perf_counter() - t0)
    cpu_s = float(np.median(times))
    sum_nrk = int(o_nrk.astype(np.int64).sum())
    # single-thread leg (1 thread and all cores): every 8th row of the same frame
    t0 = time.perf_counter()
    _, _, s_nrk, _ = oracle.render_rows(cu, U, sky, W, H, cap, scene.scene_flags, 0, H, threads=1, row_step=8)
    one_s = time.perf_counter() - t0
    cpu_baseline = {"value": round(W * H / cpu_s / 1e6, 4), "unit": "Mpix/s", "cores": threads, "kind": "port",
                    "sample": f"the full {W}x{H} cap-{cap} frame, x{len(times)} (median {cpu_s:.2f} s): C oracle "
                              f"(oracle/bh_oracle.c, gcc -O2 -ffp-contract=off), OpenMP {threads} threads",
                    "n_rk_per_s": round(sum_nrk / cpu_s, 1),
                    "single_thread": {"value": round(s_nrk.size / one_s / 1e6, 4), "unit": "Mpix/s",
                                      "n_rk_per_s": round(int(s_nrk.astype(np.int64).sum()) / one_s, 1),
                                      "sample": f"every 8th row of the frame ({s_nrk.size} px, {one_s:.2f} s), 1 thread"},
                    "host": {"cpu": _cpu_model(), "nproc": os.cpu_count(),
                             "affinity": len(os.sched_getaffinity(0))}}
    c32 = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
    nrk = torch.empty((H, W), dtype=torch.int16, device=dev)
    fate = torch.empty((H, W), dtype=torch.uint8, device=dev)
    scene.render(c32, None, fmt=bh.BH_OUT_RGBA32F, stream=stream, dbg_n_rk=nrk, dbg_fate=fate, schedule=sched)
    torch.cuda.synchronize()
    gc, gn, gf = c32.cpu().numpy(), nrk.cpu().numpy().view(np.uint16), fate.cpu().numpy()
    match = (gf == o_fate) & (gn == o_nrk)
    d = np.abs(gc[..., :3] - o_col[..., :3]).max(axis=-1)
    parity = {"vs": "oracle/bh_oracle.c (normative restatement of src/black_hole_maybe.wgsl; parity unpinned "
                    "against the WGSL itself, which cannot run here)",
              "pixels": int(match.size), "fate_nrk_match": round(float(match.mean()), 7),
              "max_abs_delta": float(d.max()), "max_abs_delta_fate_matched": float(d[match].max()),
              "bit_exact": bool(np.array_equal(gc.view(np.uint32), o_col.view(np.uint32))),
              "tolerance": 1e-4, "math": args.math}
    return cpu_baseline, parity


if __name__ == "__main__":
    main()
