"""Multi-rank host logic on CPU with the gloo backend (world size 2 and 3): every rank packs its
(tx + 3*ty) % world share of 8x8 tiles, one gather brings them to rank 0, and the unpacked frame
is the full frame.  Same functions as bench.py's N>1 path; on GPUs the collective is RCCL and the
unpack is the bh_tiles_unpack kernel (covered by tests/test_gpu_parity.py)."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, q):
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist
    from black_hole_ray_marching_amd import multigpu
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stride = multigpu.packed_stride(W, H, world)
        packed = torch.full((stride * 64, 2), -1, dtype=torch.int64)
        lane = torch.arange(64)
        for t, (tx, ty) in enumerate(multigpu.shard_tiles(W, H, rank, world)):
            packed[t * 64 + lane, 0] = int(tx) * 8 + (lane & 7)
            packed[t * 64 + lane, 1] = int(ty) * 8 + (lane >> 3)
        got = multigpu.gather_packed(packed, rank, world)
        # timing protocol of bench.py: max over ranks
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            allp = torch.cat(got).numpy()
            frame = multigpu.unpack_tiles_numpy(allp, W, H, world, stride)
            yy, xx = np.mgrid[0:H, 0:W]
            ok = bool(np.array_equal(frame[..., 0], xx) and np.array_equal(frame[..., 1], yy))
            q.put((ok, float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H", [(2, 100, 52), (3, 64, 40)])
def test_gather_and_unpack_full_frame(world, W, H):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, tmax = q.get(timeout=5)
    assert ok and tmax == float(world)


def _pipeline_worker(rank, world, port, W, H, K, q):
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist
    from black_hole_ray_marching_amd import multigpu
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stride = multigpu.packed_stride(W, H, world)
        tiles = multigpu.shard_tiles(W, H, rank, world)
        lane = torch.arange(64)
        seen = []

        def on_frame(i, gathered):
            frame = multigpu.unpack_tiles_numpy(gathered.numpy(), W, H, world, stride)
            yy, xx = np.mgrid[0:H, 0:W]
            seen.append((i, bool(np.array_equal(frame[..., 0], xx) and np.array_equal(frame[..., 1], yy)
                                  and (frame[..., 2] == i).all())))

        pipe = multigpu.GatherPipeline(lambda: torch.full((stride * 64, 3), -1, dtype=torch.int64),
                                       rank, world, on_frame, depth=2)
        for i in range(K):
            buf = pipe.buffer(i)          # "render" frame i: pixel coordinates + frame number
            for t, (tx, ty) in enumerate(tiles):
                buf[t * 64 + lane, 0] = int(tx) * 8 + (lane & 7)
                buf[t * 64 + lane, 1] = int(ty) * 8 + (lane >> 3)
                buf[t * 64 + lane, 2] = i
            pipe.submit(i)
        pipe.drain()
        if rank == 0:
            q.put(seen)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H", [(2, 100, 52), (3, 64, 40)])
def test_gather_pipeline_delivers_every_frame_in_order(world, W, H):
    """bench.py's N>1 loop: double-buffered packed tiles, async gather per frame, rank-0 unpack."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, K = _free_port(), 5
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, W, H, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    seen = q.get(timeout=5)
    assert seen == [(i, True) for i in range(K)]
