#!/usr/bin/env python3
"""Headline benchmark: Mpix/s of the geodesic ray-march at 4096x2048 with a 512 RK-step cap
(BASELINE.json configs[2]) and the max |delta pixel| against the CPU oracle (the normative WGSL
restatement, oracle/bh_oracle.c).

A "step" is one batch of the offline renderer: ONE bh_render_frames launch of D frames of the
camera path (D = --frames-per-launch, 32 at N = 1 for the headline; every frame is a full pass of the
hot path, Scene::render -> the HIP march kernel, over the synthetic frame, the sky already resident in
HBM).  `value` = frames x W x H / the timed region's wall time; `ms_per_step` is per batch and
`ms_per_frame` per frame.  Default arithmetic: BH_MATH_EXACT, the bit-exact path (the only one that can
meet |delta| < 1e-4); RGBA16F col + blackout targets as north_star asks.  Besides the
headline the line carries `single_frame` (one bh_render per frame, the reference's one Scene::render
per redraw, src/state.rs:270-279) and `orbit` (every frame its own camera), untimed for `value`, and
`clock`: the shader clock measured inside the timed launches (bh_set_clock_probe).

Workloads (--workload):
  strong   (default) north_star's fixed 4096x2048 frame, split over the N GPUs (strong scaling; at
           N=1 this is the headline, BASELINE configs[2]);
  config4  BASELINE configs[3]: the fixed 8192x4096 frame split over the N GPUs (8 in the config);
  weak     ~8.4 Mpix per GPU at aspect 2:1 (the frame grows with N).
N>1: one process per GPU (torch.distributed, RCCL).  Each rank renders its (tx + 3*ty) % N share of
8x8 tiles of the batch's D frames in BH_LAYOUT_TILES_RGBM (RGB planes + the blackout mask word: 6.125 B
per RGBA16F pixel), the batch's shards are gathered to rank 0 (one collective per batch, overlapped with
the next batch's render), and rank 0 unpacks BOTH targets, col and blackout_col, row-major.  Every timed
step includes render, gather and unpack; the line carries a per-rank breakdown (`ranks`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload strong|config4|weak]

Without torchrun, `--gpus N` (N > 1) starts its own N ranks (child processes, before anything
touches a GPU) and exits non-zero unless all N ranks finish; the ranks never fall back to fewer GPUs.
"""
from __future__ import annotations

import argparse
import datetime
import gc
import json
import os
import socket
import subprocess
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Mpix/s at 4096×2048, 512 RK steps; max |Δpixel| vs WGSL ref"
F_STEP = {3: 209, 0: 159}  # flop-equivalents per completed RK step (surfaces on / off), SURVEY §8d
PEAK_FP32_TFLOPS = 157.3   # MI355X FP32 vector peak (MI355X_MICROARCH.md chip table)
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec

# tile rows in flight of rank 0's unpack (bh_tiles_unpack_rgbm rows_in_flight)
UNPACK_ROWS_IN_FLIGHT = 64

WORKLOADS = {"strong": (4096, 2048), "config4": (8192, 4096)}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # a step is one batch (one launch of D frames): 20 x 32 = 640 timed frames at the headline
    p.add_argument("--steps", type=int, default=20)
    # 10 warm-up batches (320 frames, ~0.2 s): past the GPU clock's ~30 ms ramp under load
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--settle-ms", type=float, default=0.0,
                   help="optional untimed power-state settle before the warm-up: full launches of the workload "
                        "for this many ms (DESIGN.md §6); 0 = none (the warm-up batches cover the clock ramp)")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the single_frame / orbit legs (N = 1) that follow the timed region")
    p.add_argument("--workload", choices=["strong", "config4", "weak"], default="strong")
    p.add_argument("--config", type=int, choices=[1, 2, 3, 4, 5], default=0,
                   help="BASELINE.json configs[N-1]: 1 = 256x256 cap 64 no surfaces camera A, 2 = 1920x1080 cap 256 "
                        "camera B, 3 = the headline, 4 = 8192x4096 cap 512 split over the N GPUs, 5 = 4096x2048 cap "
                        "1000 camera C (sets frame, cap, camera and scene; other flags still apply)")
    p.add_argument("--math", choices=["exact", "fast"], default="exact")
    p.add_argument("--schedule", choices=["tile", "tile-static", "pair", "persistent"], default="tile")
    p.add_argument("--variant", choices=["auto", "issue", "latency"], default="auto",
                   help="exact math: build of the march kernels (auto: per frame, include/bh_render.h)")
    p.add_argument("--fmt", choices=["rgba16f", "rgba32f", "bgra8"], default="rgba16f")
    p.add_argument("--width", type=int, default=0)
    p.add_argument("--height", type=int, default=0)
    p.add_argument("--max-iters", type=int, default=512)
    p.add_argument("--camera", choices=["A", "B", "C"], default="A")
    p.add_argument("--orbit-deg", type=float, default=0.2, help="--camera-path orbit: degrees per frame")
    p.add_argument("--camera-path", choices=["fixed", "orbit"], default="fixed",
                   help="orbit: frame i's camera is the chosen one rotated about the y axis by i x 0.2 degrees "
                        "(an offline camera path: every frame of a multi-frame launch has its own camera)")
    p.add_argument("--surfaces", choices=["on", "off"], default="on",
                   help="off = scene_flags 0 (no disc, no markers: BASELINE config 1's scene)")
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline / parity leg")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may use")
    p.add_argument("--cpu-reps", type=int, default=3)
    p.add_argument("--graph", action="store_true",
                   help="N=1: capture one frame's bh_render (order kernel + march) in a HIP graph and replay it")
    p.add_argument("--verify-gather", action="store_true",
                   help="N>1: rank 0 compares both assembled targets with its own full-frame render (bitwise)")
    p.add_argument("--frames-per-launch", type=int, default=0,
                   help="frames rendered by one bh_render_frames launch (1..256; 0 = auto, DESIGN.md §5 item 9)")
    p.add_argument("--root-ratio", default="calibrate",
                   help="N>1: rank 0's tile share relative to each other rank's (it also unpacks every frame, and its "
                        "own tiles cross no link): 'calibrate' (default: the fastest of a few candidates, measured "
                        "before the warm-up), 'auto' (multigpu.auto_root_ratio) or a number; 1 = the plain "
                        "(tx + 3ty) %% N interleave")
    p.add_argument("--unpack-priority", choices=["high", "normal"], default="high",
                   help="N>1: the priority of rank 0's unpack stream (high: overlaps the next batch's render)")
    p.add_argument("--transport", choices=["auto", "rgbm", "rgbm14"], default="auto",
                   help="N>1 shard layout: BH_LAYOUT_TILES_RGBM (6.125 B/pixel of RGBA16F) or BH_LAYOUT_TILES_RGBM14 "
                        "(5.375: the fp16 channels in [0, 1] take 14 bits); auto = rgbm14 for rgba16f")
    p.add_argument("--deadline-s", type=float, default=420.0,
                   help="self-launched N>1 run: stop every rank and exit non-zero after this many seconds "
                        "(below the driver's 600 s limit, so that its error line is what the driver records; "
                        "a healthy 8-rank run takes well under a minute)")
    p.add_argument("--stall-s", type=float, default=90.0,
                   help="per-rank watchdog: a rank that makes no progress (no launch issued, no batch "
                        "synchronised) for this many seconds -- a kernel or a collective that does not "
                        "return -- exits with status 125, and the launcher stops the others; 0 = off")
    p.add_argument("--pg-timeout-s", type=float, default=120.0,
                   help="torch.distributed process-group timeout (init and every collective)")
    p.add_argument("--plumbing", action="store_true",
                   help="no GPU: the N-rank launch, gather pipeline and RGBM unpack on CPU (gloo) with "
                        "synthetic shards (tests only; prints no measurement)")
    p.add_argument("--rccl-dry-run", action="store_true",
                   help="--gpus 1 only: run the N>1 code path with one rank -- an RCCL (nccl backend) process "
                        "group of world size 1, RGBM shard render, pipelined dist.gather, rank-0 unpack -- to "
                        "check the collectives on a 1-GPU box (development; not the N=1 measurement)")
    return p.parse_args(argv)


CAMERAS = {"A": ((0.0, 0.0, -20.0), (0.0, 0.0, 0.0)),   # == Scene::new's camera (src/scene.rs:68-76)
           "B": ((0.0, 3.0, -20.0), (0.0, 0.0, 0.0)), "C": ((0.0, 6.0, -12.0), (0.0, 0.0, 0.0))}
ORBIT_DEG_PER_FRAME = 0.2


def orbit_camera(bh, camera: str, i: int, W: int, H: int, deg: float = ORBIT_DEG_PER_FRAME):
    """Camera uniform of frame i of the orbit path: the named camera's position rotated about the y axis
    through the black hole by i * deg degrees, looking at the origin."""
    pos, target = CAMERAS[camera]
    a = np.radians(deg * i)
    p = (pos[0] * np.cos(a) + pos[2] * np.sin(a), pos[1], -pos[0] * np.sin(a) + pos[2] * np.cos(a))
    cu = bh.CameraUniform()
    cu.update(bh.Camera.look_at(tuple(float(v) for v in p), target, W, H))
    return cu


# ---- rank launcher (no torchrun) --------------------------------------------------------------------

def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class Watchdog:
    """Ends this rank when it stops making progress: a daemon thread checks once a second that beat() was
    called within `stall_s` seconds and otherwise prints what the rank was doing and exits the process with
    status 125 (os._exit: the main thread may be blocked inside a HIP synchronise or a collective that never
    returns).  The process-group timeout covers collectives only; this also covers a rank stuck in a kernel
    or a calibration loop.  The launcher then stops the other ranks."""

    EXIT = 125

    def __init__(self, rank: int, stall_s: float):
        self.rank, self.stall_s = rank, stall_s
        self.t, self.what = time.monotonic(), "start"
        self._done = threading.Event()
        if stall_s > 0:
            threading.Thread(target=self._run, name="bench-watchdog", daemon=True).start()

    def beat(self, what: str | None = None) -> None:
        self.t = time.monotonic()
        if what:
            self.what = what

    def stop(self) -> None:
        self._done.set()

    def _run(self) -> None:
        while not self._done.wait(1.0):
            idle = time.monotonic() - self.t
            if idle > self.stall_s:
                print(f"bench: rank {self.rank}: no progress for {idle:.0f} s in '{self.what}' (a kernel or "
                      f"collective that does not return); exiting with status {self.EXIT}", file=sys.stderr,
                      flush=True)
                os._exit(self.EXIT)


_WD = Watchdog(0, 0.0)  # replaced per rank by main() / plumbing()


def beat(what: str | None = None) -> None:
    _WD.beat(what)


def _stop(procs, live, grace_s: float = 10.0) -> None:
    """SIGTERM the live ranks (by PID), then SIGKILL whatever is still running after `grace_s`."""
    for q in live:
        procs[q].terminate()
    end = time.monotonic() + grace_s
    for q in live:
        try:
            procs[q].wait(timeout=max(0.0, end - time.monotonic()))
        except subprocess.TimeoutExpired:
            procs[q].kill()
            procs[q].wait()


def launch_ranks(n: int, argv: list[str], deadline_s: float) -> int:
    """Start this script as N ranks (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their env, as
    torchrun sets them) and wait for all of them.  The parent never touches a GPU (it does not even
    import torch), so the children are plain fork+exec of an uninitialised process.  If any rank
    fails, the others are terminated (by PID) and the exit status is non-zero.  If the ranks have not
    all finished `deadline_s` after the start (a wedged collective, a hung rank), every rank is stopped
    and the launcher prints one {"error": ...} line and exits non-zero: a hang costs the deadline, not
    the driver's whole time limit."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *argv], env=env))
    rc = 0
    live = set(range(n))
    t_end = time.monotonic() + deadline_s
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                why = " (its watchdog: no progress)" if c == Watchdog.EXIT else ""
                print(f"bench: rank {r} exited with status {c}{why}; stopping the other ranks", file=sys.stderr)
                print(json.dumps({"error": f"rank {r} of {n} exited with status {c}{why}; all ranks stopped",
                                  "n_gpus": n}), flush=True)
                _stop(procs, live)
                live.clear()
        if live and time.monotonic() > t_end:
            print(json.dumps({"error": f"deadline: ranks {sorted(live)} of {n} still running after {deadline_s:.0f} s; "
                                       "all ranks stopped", "n_gpus": n}), flush=True)
            _stop(procs, live)
            return 124
        time.sleep(0.05)
    return rc


def root_weights(args, n: int):
    """The weighted partition of an N>1 run (rank 0 lighter, it also unpacks), or None for the plain
    interleave (N = 1 or --root-ratio 1)."""
    if n == 1:
        return None
    from black_hole_ray_marching_amd import multigpu
    # 'calibrate' measures (bench main); without a GPU (plumbing) it falls back to the model's ratio
    ratio = multigpu.auto_root_ratio(n) if args.root_ratio in ("auto", "calibrate") else float(args.root_ratio)
    w = multigpu.root_weights(n, ratio)
    return None if len(set(w)) == 1 else w


# ---- host facts for the CPU baseline ----------------------------------------------------------------

def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpus() -> dict:
    """CPUs this process may run on: the affinity mask, and a cgroup v2 CPU quota if one is set
    (a quota of q CPUs caps the host work per second at q cores, whatever the affinity says)."""
    info = {"cpu": _cpu_model(), "nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "cgroup_quota_cpus": None, "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            info["cgroup_quota_cpus"] = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return info


# ---- CPU plumbing rehearsal (tests) ------------------------------------------------------------------

def plumbing(args, rank: int, n: int) -> int:
    """The N>1 data path without a GPU: every rank packs synthetic BH_LAYOUT_TILES_RGBM shards of a
    small RGBA16F frame (multigpu.pack_rgbm_numpy, the march kernel's store), the GatherPipeline brings
    each frame to rank 0 over gloo, and rank 0 restores col and blackout_col (unpack_rgbm_numpy, the
    bh_tiles_unpack_rgbm mirror) and checks them against the frame."""
    import torch
    import torch.distributed as dist

    from black_hole_ray_marching_amd import multigpu
    global _WD
    if n > 1:
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=args.pg_timeout_s))
    _WD = Watchdog(rank, args.stall_s)
    if os.environ.get("BH_PLUMBING_FAIL_RANK") == str(rank):  # test hook: a rank that dies mid-run
        raise SystemExit(f"plumbing: rank {rank} failing on request")
    if os.environ.get("BH_PLUMBING_HANG_RANK") == str(rank):  # test hook: a rank that hangs mid-run
        beat("the hang test hook")
        while True:
            time.sleep(1.0)
    W, H = (args.width or 100), (args.height or 52)
    weights = root_weights(args, n)
    stride = multigpu.packed_stride(W, H, n, weights)
    p14 = args.transport != "rgbm"  # the frame is RGBA16F
    tb = multigpu.RGBM14_TILE_BYTES if p14 else multigpu.rgbm_tile_bytes(1)
    yy, xx = np.mgrid[0:H, 0:W]

    def frame(i):
        c = np.stack([(xx % 7) * 0.25, (yy % 5) * 0.25, ((xx + yy + i) % 3) * 0.5, np.ones_like(xx)], -1)
        c32 = c.astype(np.float32)
        zero = ((c32[..., 0] * c32[..., 0] + c32[..., 1] * c32[..., 1]) + c32[..., 2] * c32[..., 2]) < 1.0
        return c32.astype(np.float16), zero

    ok = []

    def on_frame(i, gathered):
        if p14:
            col, bo = multigpu.unpack_rgbm14_numpy(gathered.numpy(), W, H, n, stride, weights)
        else:
            col, bo = multigpu.unpack_rgbm_numpy(gathered.numpy(), W, H, n, stride, np.float16, 1.0, weights)
        want, zero = frame(i)
        want_bo = want.copy()
        want_bo[zero, :3] = 0
        ok.append(bool(np.array_equal(col.view(np.uint16), want.view(np.uint16))
                       and np.array_equal(bo.view(np.uint16), want_bo.view(np.uint16))))

    pipe = multigpu.GatherPipeline(lambda: torch.zeros((stride, tb), dtype=torch.uint8), rank, n, on_frame)
    for i in range(args.steps):
        beat(f"plumbing frame {i}")
        c, z = frame(i)
        pack = multigpu.pack_rgbm14_numpy if p14 else multigpu.pack_rgbm_numpy
        pipe.buffer(i).copy_(torch.from_numpy(pack(c, z, rank, n, stride, weights)))
        pipe.submit(i)
    pipe.drain()
    world = dist.get_world_size() if n > 1 else 1
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Mpix/s", "n_gpus": n, "steps": args.steps,
                          "data": "plumbing (CPU, gloo, synthetic RGBM shards; no GPU, not a measurement)",
                          "transport": "rgbm14" if p14 else "rgbm",
                          "world_size": world, "backend": dist.get_backend() if n > 1 else None,
                          "partition_weights": weights,
                          "frames_checked": len(ok), "gather_verified_bit_exact": bool(ok) and all(ok)}))
    if n > 1:
        dist.barrier()
        dist.destroy_process_group()
    _WD.stop()
    return 0 if (rank != 0 or (len(ok) == args.steps and all(ok))) else 3


# ---- the measurement ---------------------------------------------------------------------------------

BASELINE_CONFIGS = {  # BASELINE.json configs -> bench flags (SURVEY §8d cameras)
    1: dict(width=256, height=256, max_iters=64, camera="A", surfaces="off"),
    2: dict(width=1920, height=1080, max_iters=256, camera="B"),
    3: dict(max_iters=512, camera="A"),
    4: dict(workload="config4", max_iters=512, camera="A"),
    5: dict(max_iters=1000, camera="C"),
}


def apply_config(args):
    """--config N: BASELINE.json configs[N-1]'s frame, cap, camera and scene."""
    for k, v in BASELINE_CONFIGS.get(args.config, {}).items():
        setattr(args, k, v)
    return args


def main() -> int:
    argv = sys.argv[1:]
    args = apply_config(parse(argv))
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, argv, args.deadline_s)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}: refusing to measure a different N")
    n = world
    if args.rccl_dry_run and n != 1:
        raise SystemExit("--rccl-dry-run runs one rank: use --gpus 1")
    sharded = n > 1 or args.rccl_dry_run  # the N>1 code path (shards, gather, unpack)
    if args.plumbing:
        return plumbing(args, rank, n)

    import torch
    import torch.distributed as dist

    import black_hole_ray_marching_amd as bh
    from black_hole_ray_marching_amd import multigpu

    # BH_BENCH_REHEARSAL=1 (development only, never set by the driver): all ranks share cuda:0 and
    # the gloo backend, to exercise the N>1 path (sharding, pipelined gather, unpack) on a 1-GPU box
    rehearsal = os.environ.get("BH_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    elif torch.cuda.device_count() < n:  # counting devices does not initialise the GPU
        raise SystemExit(f"--gpus {n}: only {torch.cuda.device_count()} GPUs visible")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if sharded:
        if args.rccl_dry_run and "MASTER_ADDR" not in os.environ:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
        # an explicit timeout: a wedged rendezvous or collective on the 8-rank node raises instead of
        # waiting forever (the launcher's deadline stops what it cannot)
        pg_timeout = datetime.timedelta(seconds=args.pg_timeout_s)
        if rehearsal:
            dist.init_process_group("gloo", timeout=pg_timeout)
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout)
        if dist.get_world_size() != n:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, expected {n}")
    global _WD
    _WD = Watchdog(rank, args.stall_s)
    beat("scene setup")

    if args.width and args.height:
        W, H = args.width, args.height
        workload = "custom"
    elif args.workload == "weak":
        W, H = multigpu.weak_scaling_frame(n)
        workload = "weak"
    else:
        W, H = WORKLOADS[args.workload]
        workload = args.workload
    scaling = "weak" if workload == "weak" else "strong"
    cap = args.max_iters
    fmt = {"rgba16f": bh.BH_OUT_RGBA16F, "rgba32f": bh.BH_OUT_RGBA32F, "bgra8": bh.BH_OUT_BGRA8_SRGB}[args.fmt]
    ch_dtype = {bh.BH_OUT_RGBA16F: torch.float16, bh.BH_OUT_RGBA32F: torch.float32,
                bh.BH_OUT_BGRA8_SRGB: torch.uint8}[fmt]
    bpp = bh.BYTES_PER_PIXEL[fmt]
    math_mode = bh.BH_MATH_EXACT if args.math == "exact" else bh.BH_MATH_FAST
    sched = {"tile": bh.BH_SCHED_TILE, "tile-static": bh.BH_SCHED_TILE | bh.BH_SCHED_FLAG_STATIC_ORDER,
             "pair": bh.BH_SCHED_PAIR, "persistent": bh.BH_SCHED_PERSISTENT}[args.schedule]
    sched |= {"auto": 0, "issue": bh.BH_SCHED_FLAG_ISSUE_ORDER, "latency": bh.BH_SCHED_FLAG_LATENCY}[args.variant]
    if sharded and args.schedule == "persistent":
        raise SystemExit("N>1 ships BH_LAYOUT_TILES_RGBM shards: tile or pair schedule only")

    sky = bh.synthetic_sky(4096, 2048)
    flags = bh.BH_SCENE_DEFAULT if args.surfaces == "on" else 0
    scene = bh.Scene(W, H, sky=sky, device=local, max_iters=cap, math=math_mode, scene_flags=flags)
    if args.camera != "A":
        scene.update(bh.Camera.look_at(*CAMERAS[args.camera], W, H))
    stream = torch.cuda.current_stream(dev)

    D = args.frames_per_launch or auto_frames_per_launch(n, W, H, cap)
    if not 1 <= D <= bh.BH_MAX_FRAMES:
        raise SystemExit(f"--frames-per-launch must be 1..{bh.BH_MAX_FRAMES}")
    weights = None
    calibration = None
    if not sharded:
        cols = [torch.empty((H, W, 4), dtype=ch_dtype, device=dev) for _ in range(D)]
        bos = [torch.empty((H, W, 4), dtype=ch_dtype, device=dev) for _ in range(D)]
        shard = dict(layout=bh.BH_LAYOUT_ROWMAJOR)
        my_tiles = ((W + 7) // 8) * ((H + 7) // 8)
        my_bytes = W * H * bpp * 2
        pipe = None
        batches = [scene.prepare_frames(cols, bos, fmt=fmt, schedule=sched, **shard)]
    else:
        p14 = args.transport == "rgbm14" or (args.transport == "auto" and fmt == bh.BH_OUT_RGBA16F)
        if p14 and fmt != bh.BH_OUT_RGBA16F:
            raise SystemExit("--transport rgbm14 packs rgba16f only")
        layout = bh.BH_LAYOUT_TILES_RGBM14 if p14 else bh.BH_LAYOUT_TILES_RGBM
        ufmt = fmt | bh.BH_UNPACK_RGBM14 if p14 else fmt  # the unpack's format argument
        tb = bh.tile_bytes(layout, fmt)
        frame_cols = [torch.empty((H, W, 4), dtype=ch_dtype, device=dev) for _ in range(D)] if rank == 0 else None
        frame_bos = [torch.empty((H, W, 4), dtype=ch_dtype, device=dev) for _ in range(D)] if rank == 0 else None
        # rank 0's unpack stream: high priority so that its workgroups take CU slots as the next batch's
        # render waves retire instead of queueing behind the whole render
        side = torch.cuda.Stream(dev, priority=-1 if args.unpack_priority == "high" else 0)

        class Rig:
            """The N>1 data path for one tile partition: each rank renders its share of the batch's D
            frames, col only (blackout target None == Option::None: its per-pixel decision travels as the
            RGBM mask), into one packed buffer; batch i's gather to rank 0 (all D frames in one collective)
            overlaps batch i+1's render; rank 0 unpacks every frame's col and blackout_col on a side stream."""

            def __init__(self, weights):
                # always a partition, equal weights included: its tile list (one load per wave) is cheaper
                # than the plain interleave's per-wave shard walk (4.48 vs 4.72 ns per tile at N = 8, D = 16)
                self.weights = weights
                self.part = bh.Partition(W, H, weights or [20] * n, device=local)
                self.stride = max(self.part.counts) if self.part else multigpu.packed_stride(W, H, n)
                self.my_tiles = self.part.counts[rank] if self.part else bh.shard_tile_count(W, H, rank, n)
                self.shard = dict(layout=layout, shard_index=rank, shard_count=n)
                if self.part:
                    self.shard["partition"] = self.part
                self.launch_frames = {}
                self.pipe = multigpu.GatherPipeline(
                    lambda: torch.empty((D * self.stride, tb), dtype=torch.uint8, device=dev), rank, n, self.on_frame,
                    side_stream=side, collective=True if args.rccl_dry_run else None, timing=True)
                self.batches = [scene.prepare_frames([buf[f * self.stride:(f + 1) * self.stride] for f in range(D)],
                                                     None, fmt=fmt, schedule=sched, **self.shard)
                                for buf in (self.pipe.buffer(k) for k in range(self.pipe.depth))]

            def close(self):
                """Free this candidate's buffers now: on_frame (a bound method) held by the pipeline is a
                reference cycle, and its receive buffers and prepared batches would otherwise stay
                allocated until the cyclic GC happens to run."""
                self.pipe.on_frame = None
                self.pipe = self.batches = self.part = None
                gc.collect()
                torch.cuda.empty_cache()

            def on_frame(self, i, gathered):  # issued on the pipeline's side stream (current stream here)
                # gathered: (n * D * stride, tb), rank k's block of D frames at k * D * stride
                st = self.stride
                for f in range(self.launch_frames.pop(i)):
                    if self.part:
                        bh.tiles_unpack_rgbm_partition(gathered[f * st:], frame_cols[f], frame_bos[f], self.part, D * st,
                                                       ufmt, stream=torch.cuda.current_stream(dev),
                                                       rows_in_flight=UNPACK_ROWS_IN_FLIGHT)
                    else:
                        bh.tiles_unpack_rgbm(gathered[f * st:], frame_cols[f], frame_bos[f], W, H, n, D * st, ufmt,
                                             stream=torch.cuda.current_stream(dev), rows_in_flight=UNPACK_ROWS_IN_FLIGHT)

            def step(self, k):  # one untimed batch (render + exchange), k = its pipeline index
                beat(f"calibration batch {k}")
                self.batches[k % len(self.batches)].render(n=D, stream=stream)
                self.launch_frames[k] = D
                self.pipe.submit(k)

        if args.root_ratio == "calibrate" and n > 1:
            # rank 0's share, measured: the batch time of a few candidate partitions --
            # rank 0 renders less when its unpack binds, more when the xGMI ingress of the others' shards
            # binds (its own tiles cross no link) -- untimed, before the warm-up; every rank takes rank 0's pick
            ratios = sorted({round(multigpu.auto_root_ratio(n), 3), 0.4, 0.55, 0.7, 0.85, 1.0, 1.15, 1.3})
            ms = []
            for r in ratios:
                rig = Rig(multigpu.root_weights(n, r) if r != 1.0 else None)
                for k in range(CALIBRATE_WARM):
                    rig.step(k)
                rig.pipe.drain()
                torch.cuda.synchronize(dev)
                dist.barrier()
                t_c = time.perf_counter()
                for k in range(CALIBRATE_WARM, CALIBRATE_WARM + CALIBRATE_STEPS):
                    rig.step(k)
                rig.pipe.drain()
                torch.cuda.synchronize(dev)
                dist.barrier()
                ms.append((time.perf_counter() - t_c) / CALIBRATE_STEPS * 1e3)
                rig.close()
                del rig
            pick = [ratios[int(np.argmin(ms))]]
            dist.broadcast_object_list(pick, src=0)
            weights = multigpu.root_weights(n, pick[0]) if pick[0] != 1.0 else None
            calibration = {"root_ratios": ratios, "ms_per_batch": [round(x, 4) for x in ms], "chosen": pick[0],
                           "batches_each": f"{CALIBRATE_WARM} warm + {CALIBRATE_STEPS} timed (untimed for value)"}
        else:
            weights = root_weights(args, n)
        rig = Rig(weights)
        part, stride, shard, pipe, batches = rig.part, rig.stride, rig.shard, rig.pipe, rig.batches
        launch_frames = rig.launch_frames
        my_tiles = rig.my_tiles
        my_bytes = my_tiles * tb + (2 * W * H * bpp if rank == 0 else 0)

    launch_no = [0]
    frame_no = [0]   # frames launched so far (the orbit path's frame index)
    orbit = {}       # frame index -> CameraUniform, built outside the timed region

    def cams(nf, path=None):
        if (path or args.camera_path) == "fixed":
            return None
        return [orbit[frame_no[0] + f] for f in range(nf)]

    def launch(nf, path=None, **kw):
        """One bh_render_frames launch of nf <= D frames (this scene's camera, or the orbit path's); with
        debug outputs (kw) an unprepared call."""
        if not kw:
            batches[launch_no[0] % len(batches)].render(n=nf, cameras=cams(nf, path), stream=stream)
        elif pipe is None:
            scene.render_frames(cols[:nf], bos[:nf], cameras=cams(nf, path), fmt=fmt, stream=stream, schedule=sched,
                                **shard, **kw)
        else:
            buf = pipe.buffer(launch_no[0])
            scene.render_frames([buf[f * stride:(f + 1) * stride] for f in range(nf)], None, cameras=cams(nf, path),
                                fmt=fmt, stream=stream, schedule=sched, **shard, **kw)

    extra = not (args.no_extra or sharded or args.graph)
    n_orbit_frames = (args.warmup + args.steps) * D if args.camera_path == "orbit" else 0
    if extra:
        # _leg's two passes + the untimed one (orbit), and the one-frame orbit leg's two passes
        n_orbit_frames = max(n_orbit_frames, 2 * EXTRA_ORBIT_LAUNCHES * D + D, 2 * EXTRA_SINGLE_FRAMES + 1)
    if n_orbit_frames:
        if args.graph:
            raise SystemExit("--graph replays one launch's cameras: use --camera-path fixed")
        orbit.update({i: orbit_camera(bh, args.camera, i, W, H, args.orbit_deg) for i in range(n_orbit_frames)})

    graph = None
    if args.graph and not sharded:
        # the temporal-order state is per (geometry, shard, stream): render once on the capture stream
        # (allocating that state), then capture on the same stream; replays run there too
        cap_stream = torch.cuda.Stream(dev)
        scene.render_frames(cols, bos, fmt=fmt, stream=cap_stream, schedule=sched, **shard)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=cap_stream):
            scene.render_frames(cols, bos, fmt=fmt, stream=cap_stream, schedule=sched, **shard)
        stream = cap_stream  # the timing events bracket the replays on the stream they run on

    def render(nf):
        beat(f"launch {launch_no[0]}")
        if graph is not None and nf == D:
            with torch.cuda.stream(stream):  # replay on the capture stream (its order state)
                graph.replay()
        else:
            launch(nf)

    def exchange(nf):
        if pipe is not None:
            launch_frames[launch_no[0]] = nf
            pipe.submit(launch_no[0])
        launch_no[0] += 1
        frame_no[0] += nf

    # optional power-state settle (DESIGN.md §6 "Warm-up"; off by default: the W warm-up batches cover
    # the clock's ~30 ms ramp under load): full launches of the same workload (render only, nothing
    # exchanged, no frame index advances) until settle_ms of GPU-busy wall time has passed.
    settle_frames, t_settle = 0, time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
        render(D)
        torch.cuda.synchronize(dev)
        settle_frames += D
    settle_ms = (time.perf_counter() - t_settle) * 1e3

    # everything the timed region needs is allocated before the warm-up, so that between the last
    # warm-up launch and the first timed one the GPU idles only for the synchronize (an idle gap of a
    # millisecond costs the next launch ~10 % of its time while the clock ramps back up)
    K = args.steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    clk = torch.zeros((4, 128), dtype=torch.int64, device=dev)  # shader clock: timed region, extra legs
    for _ in range(args.warmup):
        render(D)
        exchange(D)
    if pipe is not None:
        pipe.drain()
    # the shader-clock probe counts from the next launch on (bh_set_clock_probe); clk was zeroed above
    if graph is None:
        scene.set_clock_probe(clk[0], CLOCK_STRIDE)

    # timed region: K steps = K batches of D frames; barrier + synchronize on both sides; HIP events
    # around every launch on the stream the kernel runs on (kernel duration for the roofline)
    first_timed = launch_no[0]
    if sharded:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(K):
        ev[i][0].record(stream)
        render(D)
        ev[i][1].record(stream)
        exchange(D)
    if pipe is not None:
        pipe.drain()
    torch.cuda.synchronize(dev)
    if sharded:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    scene.set_clock_probe(None)
    per_rank = [elapsed]
    if sharded:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        gl = [torch.zeros_like(t) for _ in range(n)]
        dist.all_gather(gl, t)
        per_rank = [float(x.item()) for x in gl]
        elapsed = max(per_rank)
    kern_ms = np.array([a.elapsed_time(b) for a, b in ev])       # per launch
    kern_avg_s = float(kern_ms.mean()) / 1e3                     # a launch's average duration
    kern_frame_s = kern_avg_s / D                                # launch time per frame
    clock = bh.clock_mhz(clk[0].cpu().numpy()) if graph is None else None

    ranks = None
    if sharded:
        # per-rank breakdown of the timed steps (HIP events): render = the launch on the render stream;
        # gaps = render-stream idle between consecutive launches (waiting for a gather slot / the host);
        # gather = render end -> the batch's collective complete (rank 0: every shard received);
        # unpack = rank 0's two-target unpack of the batch; drain = rank 0, last render end -> last unpack end
        tl = pipe.timeline(range(first_timed, first_timed + K))
        gaps = [ev[i][1].elapsed_time(ev[i + 1][0]) for i in range(K - 1)]
        mine = {"rank": rank, "render_ms": round(float(kern_ms.mean()), 4),
                "render_ms_min_max": [round(float(kern_ms.min()), 4), round(float(kern_ms.max()), 4)],
                "render_gap_ms": round(float(np.mean(gaps)) if gaps else 0.0, 4),
                "gather_ms": round(float(np.mean(tl["gather_ms"])), 4) if tl["gather_ms"] else None,
                "unpack_ms": round(float(np.mean(tl["unpack_ms"])), 4) if tl["unpack_ms"] else None,
                "wall_s": round(per_rank[rank] if len(per_rank) > rank else elapsed, 6),
                "clock_mhz": clock["mhz"] if clock else None}
        if rank == 0 and tl["unpack_ms"]:
            last = pipe.events.get(first_timed + K - 1, {})
            if "unpacked" in last:
                mine["drain_ms"] = round(ev[K - 1][1].elapsed_time(last["unpacked"]), 4)
        ranks = [None] * n
        dist.all_gather_object(ranks, mine)

    gather_ok = None
    beat("after the timed region")
    if args.verify_gather and sharded and rank == 0:
        # every frame of the last batch against a single-GPU render of that frame's camera
        ref_c = torch.empty((H, W, 4), dtype=ch_dtype, device=dev)
        ref_b = torch.empty((H, W, 4), dtype=ch_dtype, device=dev)
        first = frame_no[0] - D  # frame index of the last batch's first frame
        gather_ok = True
        for f in range(D):
            beat(f"verify frame {f}")
            if args.camera_path == "orbit":
                scene.render_frames([ref_c], [ref_b], cameras=[orbit[first + f]], fmt=fmt, stream=stream,
                                    schedule=sched)
            else:
                scene.render(ref_c, ref_b, fmt=fmt, stream=stream, schedule=sched)
            torch.cuda.synchronize(dev)
            gather_ok = gather_ok and bool(torch.equal(ref_c.view(torch.uint8), frame_cols[f].view(torch.uint8))
                                           and torch.equal(ref_b.view(torch.uint8), frame_bos[f].view(torch.uint8)))
        del ref_c, ref_b

    # the unfavourable cases beside the headline (N = 1, not part of `value`): one bh_render per frame
    # (the reference's one Scene::render per redraw), and an orbiting camera path (every frame its own
    # camera, so the learned dispatch order is a launch stale)
    legs = {}
    if extra:
        legs["single_frame"] = _leg(lambda: launch(1, path="fixed"), EXTRA_SINGLE_FRAMES, 1, scene, clk[1], stream, dev, W, H, torch, bh)
        frame_no[0] = 0
        launch(D, path="orbit")  # untimed: the order learns the path's start
        frame_no[0] = D

        def orbit_launch():
            launch(D, path="orbit")
            frame_no[0] += D
        legs["orbit"] = _leg(orbit_launch, EXTRA_ORBIT_LAUNCHES, D, scene, clk[2], stream, dev, W, H, torch, bh)
        legs["single_frame"]["note"] = ("one bh_render_frames(n=1) per frame, fixed camera, back to back: the "
                                        "reference's one Scene::render per redraw (src/state.rs:270-279); a "
                                        "repeated frame skips the dispatch-order build (its costs are the ones "
                                        "the order holds), so this is the static camera's best case: "
                                        "single_frame_orbit moves the camera every frame")
        frame_no[0] = 0
        launch(1, path="orbit")  # untimed: the order learns the path's start
        frame_no[0] = 1

        def orbit_single():
            launch(1, path="orbit")
            frame_no[0] += 1
        legs["single_frame_orbit"] = _leg(orbit_single, EXTRA_SINGLE_FRAMES, 1, scene, clk[3], stream, dev, W, H,
                                          torch, bh)
        legs["single_frame_orbit"].update(deg_per_frame=args.orbit_deg, note=(
            f"one bh_render_frames(n=1) per frame, camera {args.camera} orbiting the hole at {args.orbit_deg} "
            "deg/frame: the interactive redraw of a moving camera (every frame builds its dispatch order from the "
            "previous frame's costs)"))
        legs["orbit"].update(deg_per_frame=args.orbit_deg, frames_per_launch=D,
                             note=f"camera {args.camera} orbiting the hole at {args.orbit_deg} deg/frame, {D} "
                                  "frames per launch each with its own camera (the dispatch order learned from "
                                  "the previous launch's frame 0)")

    # algorithmic work of one launch: RK steps over this rank's pixels (deterministic).  sum_n_rk is
    # the loop's own count (what the reference iterates); sum_steps the updates actually executed
    # (lower by the cycle fast-forward of the tile schedule) -- the roofline uses the latter.
    px_shape = (H, W) if not sharded else (stride * 64,)  # the layout's pixel index space
    nm = 1 if args.camera_path == "fixed" else D  # orbit: every frame of a launch (own cameras), averaged
    frame_no[0] = 0
    beat("step counts")
    nrk_bufs = [torch.zeros(px_shape, dtype=torch.int16, device=dev) for _ in range(nm)]
    steps_bufs = [torch.zeros(px_shape, dtype=torch.int16, device=dev) for _ in range(nm)]
    launch(nm, dbg_n_rk=nrk_bufs, dbg_steps=steps_bufs)
    torch.cuda.synchronize(dev)
    sum_nrk = sum(int(b.cpu().numpy().view(np.uint16).astype(np.int64).sum()) for b in nrk_bufs) // nm
    sum_steps = sum(int(b.cpu().numpy().view(np.uint16).astype(np.int64).sum()) for b in steps_bufs) // nm

    if rank == 0:
        frames = K * D
        value = W * H * frames / elapsed / 1e6
        # per launch: D frames' executed steps / the launch's average duration (HIP events)
        achieved_tf = sum_steps * D * F_STEP[flags] / kern_avg_s / 1e12
        alg_bytes = int(my_bytes * D) + sky.nbytes
        achieved_gbs = alg_bytes / kern_avg_s / 1e9
        pmc = _pmc_entry(W, H, cap, args, n, D)
        mhz = clock["mhz"] if clock else None
        result = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mpix/s",
            "n_gpus": n,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 5),
            "ms_per_frame": round(elapsed / frames * 1e3, 5),
            "frames_per_s": round(frames / elapsed, 2),
            "step": f"one batch: one bh_render_frames launch of {D} frames (ms_per_step is per batch)",
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (splitmix64-seeded 4096x2048 RGBA8 sRGB sky; reference default camera)",
            "config": {
                "workload": f"{workload}: {W}x{H} frame, cap {cap} RK steps, "
                            f"{'disc+markers+sky' if flags else 'sky only (no surfaces)'}, camera {args.camera}"
                            + (f" orbiting {args.orbit_deg} deg/frame" if args.camera_path == "orbit" else "") + ", "
                            f"{args.fmt} col+blackout, {args.math} math, {D} frames per step"
                            + ("" if not sharded else
                               ", 8x8 tiles dealt by a weighted tile-list partition (bh_partition: rank k owns "
                               f"weights[k] of every sum(weights) residues of (tx+3ty), weights {weights or [20] * n}), "
                               f"{dist.get_backend() if dist.is_initialized() else 'no'} "
                               f"{'(RCCL) ' if dist.is_initialized() and dist.get_backend() == 'nccl' else ''}gather of "
                               f"{'RGBM14' if p14 else 'RGBM'} shards (RGB + blackout mask) to rank 0 overlapped "
                               "with the next batch, rank 0 unpacks col and blackout_col"
                               + (" (REHEARSAL: every rank on cuda:0 over gloo)" if rehearsal else "")),
                "baseline_config": args.config or None,
                "width": W, "height": H, "max_iters": cap, "camera": args.camera, "camera_path": args.camera_path,
                "math": args.math,
                "schedule": args.schedule, "format": args.fmt, "frames_per_launch": D,
                "parallelism": ("single GPU" + (", HIP graph replay" if graph is not None else "")) if not sharded
                               else f"tile-sharded x{n}"
                               + (f", weighted partition {weights} (rank 0 also unpacks)" if n > 1 and weights else "")
                               + (" (REHEARSAL: all ranks on cuda:0, gloo; not a measurement)" if rehearsal else "")
                               + (" (RCCL DRY RUN: the N>1 path at one rank; not the N=1 measurement)"
                                  if args.rccl_dry_run else ""),
                **({"partition_weights": weights, "tiles_per_rank_max": stride} if sharded else {}),
            },
            "kernel": {"name": f"bh::{kernel_ns(args, my_tiles, D, cap, dev)}::march_{args.schedule.split('-')[0]}_kernel<{fmt}u"
                               + ((f", {flags}u>" if flags in (0, 3) else ", 4294967295u>")  # SF: 0/3 folded, else dynamic
                                  if args.schedule.startswith("tile") else ">"),
                       "launches": K, "frames_per_launch": D, "tiles_per_frame": my_tiles,
                       "avg_ms": round(kern_avg_s * 1e3, 5), "min_ms": round(float(kern_ms.min()), 5),
                       "max_ms": round(float(kern_ms.max()), 5), "ms_per_frame": round(kern_frame_s * 1e3, 5),
                       "sum_n_rk": sum_nrk, "sum_steps": sum_steps,
                       "mean_n_rk": round(sum_nrk / (my_tiles * 64), 4), "frames_per_s": round(1.0 / kern_frame_s, 2),
                       "note": "avg/min/max over the K timed launches (HIP events on the render stream, the order "
                               "kernel included); sum_n_rk / sum_steps per frame (this rank's tiles)"},
            "clock": (dict(clock, stride=CLOCK_STRIDE,
                           note="shader clock during the timed launches: one wave in "
                                f"{CLOCK_STRIDE} of the march kernel (spread over the XCDs; per_xcd_mhz by "
                                "HW_REG_XCC_ID) reads s_memtime (shader clock) and "
                                "s_memrealtime (100 MHz) at its start and end (bh_set_clock_probe); mhz = 100 x "
                                "sum(shader ticks) / sum(100 MHz ticks) over those waves; peak_mhz is the clock "
                                "the 157.3 TFLOP/s peak assumes") | {"peak_mhz": PEAK_MHZ}) if clock else None,
            "clock_settle": {"ms": round(settle_ms, 1), "frames": settle_frames} if args.settle_ms > 0 else None,
            "roofline": {"bound": "valu", "achieved": round(achieved_tf, 3), "peak": PEAK_FP32_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved_tf / PEAK_FP32_TFLOPS, 5),
                         "frac_at_measured_clock": (round(achieved_tf / (PEAK_FP32_TFLOPS * mhz / PEAK_MHZ), 5)
                                                    if mhz else None),
                         "traffic": (round(pmc["hbm_bytes_per_launch"]) if pmc.get("hbm_bytes_per_launch") else None),
                         "valu_busy": pmc.get("valu_busy_est"),
                         "valu_lane_utilization": pmc.get("valu_lane_utilization"),
                         "pmc_source": pmc.get("source"),
                         "issue_slot_frac": round(achieved_tf / (PEAK_FP32_TFLOPS / 2), 5),
                         "note": f"{F_STEP[flags]} flop-eq per executed RK step (SURVEY §8d) x sum_steps x "
                                 "frames_per_launch / avg launch time (HIP events on the render stream); FP32 "
                                 "VALU-bound, no MFMA-shaped work; frac_at_measured_clock = achieved over the "
                                 "peak scaled to the clock measured in the timed launches (clock.mhz / "
                                 "clock.peak_mhz); traffic = HBM bytes/launch and valu_busy = VALU "
                                 "issue cycles / SIMD cycles, from the rocprofv3 PMC passes of this configuration "
                                 "named in pmc_source (profiles/pmc_traffic.json), null if none. The 157.3 TFLOP/s "
                                 "peak counts an FMA as 2 flops in every lane-cycle; the WGSL's op sequence has no "
                                 "FMA to contract (exact mode), so its ceiling is half that: issue_slot_frac = "
                                 "achieved / 78.65 (DESIGN.md §6)"},
            "roofline_hbm": {"bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": PEAK_HBM_GBS,
                             "unit": "GB/s", "frac": round(achieved_gbs / PEAK_HBM_GBS, 5),
                             "algorithmic_bytes_per_launch": alg_bytes,
                             "note": "this rank's outputs (N>1: its RGBM shard, and on rank 0 the two "
                                     "unpacked targets) + the sky texture read once"},
            **legs,
        }
        if sharded:
            result["world_size"] = dist.get_world_size()
            result["backend"] = dist.get_backend()
            result["transport"] = {"layout": "rgbm14" if p14 else "rgbm", "tile_bytes": tb,
                                   "bytes_per_pixel": round(tb / 64.0, 4), "unpack_priority": args.unpack_priority}
            result["per_rank_s"] = [round(x, 6) for x in per_rank]
            result["ranks"] = ranks
            result["partition_calibration"] = calibration
        if args.no_cpu or sharded:
            result["cpu_baseline"] = None
        else:
            beat("cpu baseline and parity")
            result["cpu_baseline"], result["parity"] = _cpu_leg(scene, sky, W, H, cap, args, dev, stream, sched, fmt)
        if gather_ok is not None:
            result["gather_verified_bit_exact"] = gather_ok
        print(json.dumps(result), flush=True)
    if sharded:
        beat("final barrier")
        dist.barrier()
        dist.destroy_process_group()
    _WD.stop()
    return 0


# extra legs after the timed region (N = 1): single-frame launches, orbit-path launches
EXTRA_SINGLE_FRAMES = 24
EXTRA_ORBIT_LAUNCHES = 4
CLOCK_STRIDE = 256   # one wave in 256 of a march launch samples the shader clock
CALIBRATE_WARM, CALIBRATE_STEPS = 2, 3   # batches per candidate partition of --root-ratio calibrate
RANK0_FRAME_BYTES = 64 << 30  # rank 0's budget for the D frames of a batch in flight (of 288 GB of HBM)
PEAK_MHZ = 2400.0    # the shader clock behind the 157.3 TFLOP/s FP32 peak (1024 SIMDs x 32 lanes x 2 x 2.4 GHz)


def _leg(fn, launches: int, frames_per_launch: int, scene, clk_row, stream, dev, W, H, torch, bh) -> dict:
    """Time `launches` calls of fn (each one launch of frames_per_launch frames) back to back, twice: first
    bare -- nothing else on the stream, as the reference's redraw loop issues its renders -- for the wall
    time (`ms_per_frame`); then with HIP events around each launch (`kernel_ms_per_frame`, from the event
    pairs) and the shader clock inside the launches (`clock_mhz`), whose event records and probe add their
    own gaps to that pass's wall time (`ms_per_frame_evented`)."""
    frames = launches * frames_per_launch
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(launches):
        beat("extra leg")
        fn()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
    scene.set_clock_probe(clk_row, CLOCK_STRIDE)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    for a, b in ev:
        beat("extra leg")
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize(dev)
    wall_ev = time.perf_counter() - t1
    scene.set_clock_probe(None)
    k = np.array([a.elapsed_time(b) for a, b in ev])
    return {"frames": frames, "ms_per_frame": round(wall / frames * 1e3, 5),
            "ms_per_frame_evented": round(wall_ev / frames * 1e3, 5),
            "kernel_ms_per_frame": round(float(k.sum()) / frames, 5),
            "mpix_s": round(W * H * frames / wall / 1e6, 3),
            "clock_mhz": bh.clock_mhz(clk_row.cpu().numpy())["mhz"]}


def kernel_ns(args, tiles: int, D: int, cap: int, dev) -> str:
    """Namespace of the march kernel bh_render runs: the fast build, or which of the two exact builds
    (bh_host.cpp march_variant_issue_order: source-order `exact` when the launch's tiles in flight,
    tiles x frames x 512 >= 384 x CUs x cap; else the scheduled `exact_lat`)."""
    if args.math != "exact":
        return "fast"
    if args.variant != "auto":
        return "exact" if args.variant == "issue" else "exact_lat"
    import torch
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    return "exact" if tiles * D * 512 >= 384 * cus * cap else "exact_lat"


def auto_frames_per_launch(n: int, W: int, H: int, cap: int) -> int:
    """Frames per launch: enough that each frame's serial tail (the few rays that march to the cap, ~0.8
    us per step alone: DESIGN.md §5) overlaps the other frames' bulk, and the per-launch cost (the order
    kernel and the gaps around it, ~16 us) is shared by many frames.  Measured (tools/probe_inflight.py,
    profiles/r02/inflight.log, profiles/r02b/frames_per_launch/; ms per frame at D = 1/2/4/8/16/32):
    4096x2048 0.658/0.633/0.621/0.609/0.606/0.602; its 1/8 shard 0.410/0.261/0.121/0.088/0.083/0.080;
    256x256 cap 64 (D = 8/16/32) 0.0095/0.0073/0.0068.  One GPU: 32 (the frames the kernel argument
    carries), and for frames of fewer than 16384 tiles enough frames for ~2^19 tiles per launch (up to
    BH_MAX_FRAMES = 256, staged through the device frame table): 256x256 cap 64 at D = 32/64/128/256
    0.00643/0.00620/0.00608/0.00604, 1920x1080 at D = 32/64/128 0.1500/0.1498/0.1492, the headline at
    D = 32/64 0.6078/0.6074 (profiles/r02c/frames_table/).  N > 1: 64 -- the last batch's gather and
    unpack cannot overlap a next render, so the pipeline drains one batch at the end of the timed region:
    with a step = one batch that is ~1/(K+1) of K steps whatever D is, while a shard's tiles get cheaper
    with longer launches (N = 8, weighted partition: 4.48 / 4.40 / 4.36 ns per tile at D = 16 / 32 / 64,
    the one-GPU frame 4.08; profiles/r04/n_gt_1/rank0_D.jsonl); the receive buffers grow with D (rank 0
    at N = 8: ~6 GB of 288)."""
    if n > 1:
        # capped by rank 0's bytes per frame in flight: its two row-major targets (RGBA16F) and
        # its share of the two receive slots (RGBM14 tiles of every rank); 64 up to ~70 Mpix frames
        tiles = ((W + 7) // 8) * ((H + 7) // 8)
        per_frame = 2 * W * H * 8 + 2 * tiles * 344
        return int(max(1, min(64, RANK0_FRAME_BYTES // per_frame)))
    tiles = ((W + 7) // 8) * ((H + 7) // 8)
    D = 32
    while D < bh_max_frames() and tiles * D < (1 << 19):
        D *= 2
    return D


def bh_max_frames() -> int:
    from black_hole_ray_marching_amd import _abi
    return _abi.BH_MAX_FRAMES


def pmc_key(W, H, cap, camera, math, schedule, fmt, n, D) -> str:
    """Key of a configuration in profiles/pmc_traffic.json (tools/pmc_summary.py writes it)."""
    return f"{W}x{H}_cap{cap}_{camera}_{math}_{schedule}_{fmt}_n{n}_D{D}"


def _pmc_entry(W, H, cap, args, n, D):
    """This configuration's entry of profiles/pmc_traffic.json (rocprofv3 PMC passes), or {}."""
    if args.camera_path != "fixed":
        return {}  # the profiled configurations are fixed-camera ones
    p = ROOT / "profiles" / "pmc_traffic.json"
    key = pmc_key(W, H, cap, args.camera, args.math, args.schedule, args.fmt, n, D)
    try:
        return json.loads(p.read_text()).get(key) or {}
    except (OSError, ValueError):
        return {}


def _cpu_leg(scene, sky, W, H, cap, args, dev, stream, sched, fmt):
    """cpu_baseline: the C oracle (gcc -O3 -ffp-contract=off, OpenMP dynamic rows) on every CPU this
    process may use, over the same full frame, `cpu_reps` times, plus a 1-thread leg on every 8th
    row; parity: the GPU frame against that oracle frame, every pixel -- in RGBA32F (the fp32
    result, bit-exact) AND in the timed format (RGBA16F: round-to-nearest-even of the oracle's fp32
    words; BGRA8: its normative sRGB encode), col and blackout_col."""
    import torch

    import black_hole_ray_marching_amd as bh
    import oracle

    host = host_cpus()
    quota = host["cgroup_quota_cpus"]
    threads = args.cpu_threads or (min(host["affinity"], max(1, int(quota))) if quota else host["affinity"])
    cu, U = scene.camera_uniform.to_bytes(), bytes(scene.uniforms.to_c())
    oracle.render_rows(cu, U, sky, W, H, cap, scene.scene_flags, 0, 64, threads=threads)  # warm-up
    times = []
    o_col = o_bo = o_nrk = o_fate = None
    for _ in range(max(1, args.cpu_reps)):
        t0 = time.perf_counter()
        o_col, o_bo, o_nrk, o_fate = oracle.render_rows(cu, U, sky, W, H, cap, scene.scene_flags, threads=threads)
        times.append(time.perf_counter() - t0)
    cpu_s = float(np.median(times))
    sum_nrk = int(o_nrk.astype(np.int64).sum())
    # single-thread leg (1 thread and all cores): every 8th row of the same frame
    t0 = time.perf_counter()
    _, _, s_nrk, _ = oracle.render_rows(cu, U, sky, W, H, cap, scene.scene_flags, 0, H, threads=1, row_step=8)
    one_s = time.perf_counter() - t0
    cpu_baseline = {"value": round(W * H / cpu_s / 1e6, 4), "unit": "Mpix/s", "cores": threads, "kind": "port",
                    "sample": f"the full {W}x{H} cap-{cap} frame, x{len(times)} (median {cpu_s:.3f} s): C oracle "
                              f"(oracle/bh_oracle.c, gcc -O3 -ffp-contract=off), OpenMP {threads} threads, "
                              "dynamic rows",
                    "n_rk_per_s": round(sum_nrk / cpu_s, 1),
                    "single_thread": {"value": round(s_nrk.size / one_s / 1e6, 4), "unit": "Mpix/s",
                                      "n_rk_per_s": round(int(s_nrk.astype(np.int64).sum()) / one_s, 1),
                                      "sample": f"every 8th row of the frame ({s_nrk.size} px, {one_s:.2f} s), 1 thread"},
                    "host": host}
    c32 = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
    b32 = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
    nrk = torch.empty((H, W), dtype=torch.int16, device=dev)
    fate = torch.empty((H, W), dtype=torch.uint8, device=dev)
    scene.render(c32, b32, fmt=bh.BH_OUT_RGBA32F, stream=stream, dbg_n_rk=nrk, dbg_fate=fate, schedule=sched)
    ch = {bh.BH_OUT_RGBA16F: torch.float16, bh.BH_OUT_RGBA32F: torch.float32, bh.BH_OUT_BGRA8_SRGB: torch.uint8}[fmt]
    tc = torch.empty((H, W, 4), dtype=ch, device=dev)
    tbo = torch.empty((H, W, 4), dtype=ch, device=dev)
    scene.render(tc, tbo, fmt=fmt, stream=stream, schedule=sched)
    torch.cuda.synchronize()
    gc, gb, gn, gf = c32.cpu().numpy(), b32.cpu().numpy(), nrk.cpu().numpy().view(np.uint16), fate.cpu().numpy()
    match = (gf == o_fate) & (gn == o_nrk)
    d = np.abs(gc[..., :3] - o_col[..., :3]).max(axis=-1)

    def expect(x):  # the timed format's bytes of an fp32 oracle image
        if fmt == bh.BH_OUT_RGBA16F:
            return x.astype(np.float16).view(np.uint8)
        if fmt == bh.BH_OUT_RGBA32F:
            return x.view(np.uint8)
        e = oracle.srgb_encode(x[..., :3])
        return np.stack([e[..., 2], e[..., 1], e[..., 0], np.full(e.shape[:2], 255, np.uint8)], -1)

    timed_ok = bool(np.array_equal(tc.cpu().numpy().view(np.uint8), expect(o_col))
                    and np.array_equal(tbo.cpu().numpy().view(np.uint8), expect(o_bo)))
    parity = {"vs": "oracle/bh_oracle.c: the normative restatement of src/black_hole_maybe.wgsl. PARITY "
                    "UNPINNED against the WGSL itself (no WGSL runtime, no reference fixtures); a real WGSL "
                    "driver's pow / atan2 / 8-bit sampler weights differ from these normative choices "
                    "(DESIGN.md §3 'Parity envelope')",
              "pixels": int(match.size), "fate_nrk_match": round(float(match.mean()), 7),
              "max_abs_delta": float(d.max()), "max_abs_delta_fate_matched": float(d[match].max()),
              # matched pixels whose ray did not run to the cap (capped rays orbit the photon sphere:
              # chaotic, any rounding difference moves where they end; tests/test_gpu_parity.py fast_stats)
              "max_abs_delta_fate_matched_uncapped": float(d[match & (o_fate != bh.BH_FATE_CAP)].max()),
              "bit_exact": bool(np.array_equal(gc.view(np.uint32), o_col.view(np.uint32))
                                and np.array_equal(gb.view(np.uint32), o_bo.view(np.uint32))),
              "timed_format": args.fmt, "timed_format_bit_exact": timed_ok,
              "tolerance": 1e-4, "math": args.math}
    return cpu_baseline, parity


if __name__ == "__main__":
    sys.exit(main())
