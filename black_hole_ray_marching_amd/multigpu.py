"""Tile-sharded frames over several GPUs (one process per GPU, torch.distributed over RCCL).

The frame is cut into 8x8 tiles; tile (tx, ty) belongs to rank (tx + 3*ty) % world (SURVEY.md
§8e: the diagonal interleave spreads the expensive photon-sphere region over all ranks; contiguous
bands would leave the centre band's owner with ~1.3x the average work).  Each rank renders its
tiles with BH_LAYOUT_TILES (or BH_LAYOUT_TILES_RGB, alpha dropped) into one contiguous buffer, the
buffers are gathered to rank 0 in a single collective (no reduction exists in this path), and rank
0 scatters them to a row-major frame with the bh_tiles_unpack(_rgb) kernel.

The reference renders one frame on one GPU (src/state.rs:255-307); this module is the multi-GPU
extension named by north_star.  The pure-Python tile math mirrors bh_common.hpp so that host logic
can be tested without a GPU.
"""
from __future__ import annotations

import numpy as np

TILE = 8


def shard_period(S: int) -> int:
    return S // 3 if S % 3 == 0 else S


def shard_row_start(ty: int, k: int, S: int) -> int:
    return (k - 3 * ty) % S


def shard_row_count(tiles_x: int, ty: int, k: int, S: int) -> int:
    st = shard_row_start(ty, k, S)
    return (tiles_x - st + S - 1) // S if st < tiles_x else 0


def shard_tile_count(width: int, height: int, k: int, S: int) -> int:
    tx, ty = (width + TILE - 1) // TILE, (height + TILE - 1) // TILE
    return sum(shard_row_count(tx, r, k, S) for r in range(ty))


def partition_owners(weights) -> list[int]:
    """Owner of each residue v of (tx + 3*ty) mod M, M = sum(weights), for a weighted partition
    (bh_host.cpp partition_owners: smooth weighted round robin)."""
    M = sum(int(w) for w in weights)
    if M <= 0 or M > 4096:
        raise ValueError("weights must sum to 1..4096")
    cw = [0] * len(weights)
    out = []
    for _ in range(M):
        best = 0
        for k, w in enumerate(weights):
            cw[k] += int(w)
            if cw[k] > cw[best]:
                best = k
        out.append(best)
        cw[best] -= M
    return out


def shard_tiles(width: int, height: int, k: int, S: int, weights=None) -> np.ndarray:
    """(n, 2) array of (tx, ty) for shard k, in its packed order (row-major over owned tiles).
    weights: a weighted partition (bh_partition_create), else the (tx + 3*ty) % S interleave."""
    tiles_x, tiles_y = (width + TILE - 1) // TILE, (height + TILE - 1) // TILE
    if weights is not None:
        own = np.array(partition_owners(weights))
        ty, tx = np.divmod(np.arange(tiles_x * tiles_y), tiles_x)
        m = own[(tx + 3 * ty) % len(own)] == k
        return np.stack([tx[m], ty[m]], -1).astype(np.int64).reshape(-1, 2)
    out = [(tx, ty) for ty in range(tiles_y) for tx in range(shard_row_start(ty, k, S), tiles_x, S)]
    return np.array(out, dtype=np.int64).reshape(-1, 2)


def root_weights(n: int, root_ratio: float, unit: int = 20) -> list[int]:
    """Weights of a partition in which rank 0 (which also unpacks every frame) takes root_ratio of
    another rank's share: [round(unit * root_ratio)] + [unit] * (n - 1)."""
    return [max(0, int(round(unit * root_ratio)))] + [unit] * (n - 1)


def auto_root_ratio(n: int) -> float:
    """Rank 0's share relative to the others' when it also unpacks both targets of every frame: the
    unpack is a fixed ~0.034 ms per 4096x2048 frame (RGBM14, HBM-bound, and it does not overlap the next
    batch's render even from a high-priority stream) while a tile renders in ~4.5 ns (tools/probe_rank0.py,
    profiles/r04/n_gt_1/): balance at (20 - w0) / (w0 + 20 (N - 1)) = U / R, i.e. r ~ 1 - 0.054 N (0.89 /
    0.78 / 0.57 at N = 2 / 4 / 8).  bench.py's calibration measures the real optimum on the node, where
    rank 0's xGMI ingress (smaller for a larger share) also counts."""
    return max(0.0, 1.0 - 0.054 * n)


def shard_tile_index(tx: int, ty: int, width: int, height: int, S: int) -> tuple[int, int]:
    """Inverse of shard_tiles (bh_common.hpp shard_tile_index): tile (tx, ty) -> (shard, local index)."""
    tiles_x = (width + TILE - 1) // TILE
    k = (tx + 3 * ty) % S
    if S == 1:
        return k, ty * tiles_x + tx
    P = shard_period(S)
    per = sum(shard_row_count(tiles_x, r, k, S) for r in range(P))
    pre = sum(shard_row_count(tiles_x, r, k, S) for r in range(ty % P))
    return k, (ty // P) * per + pre + tx // S


def packed_stride(width: int, height: int, S: int, weights=None) -> int:
    """Tiles per rank in the gather buffer (the largest shard; smaller shards are padded)."""
    if weights is not None:
        return max(len(shard_tiles(width, height, k, S, weights)) for k in range(S))
    return max(shard_tile_count(width, height, k, S) for k in range(S))


def unpack_tiles_numpy(packed: np.ndarray, width: int, height: int, S: int, stride: int) -> np.ndarray:
    """Reference (CPU) version of bh_tiles_unpack: packed (S*stride*64, C) -> (height, width, C)."""
    C = packed.shape[-1]
    out = np.zeros((height, width, C), dtype=packed.dtype)
    lane = np.arange(64)
    for k in range(S):
        for t, (tx, ty) in enumerate(shard_tiles(width, height, k, S)):
            px, py = tx * TILE + (lane & 7), ty * TILE + (lane >> 3)
            ok = (px < width) & (py < height)
            out[py[ok], px[ok]] = packed[(k * stride + t) * 64 + lane[ok]]
    return out


def planar_to_packed(planar: np.ndarray, alpha) -> np.ndarray:
    """BH_LAYOUT_TILES_RGB buffer (n_tiles, 3, 64) -> BH_LAYOUT_TILES pixels (n_tiles * 64, 4), the
    constant `alpha` (1.0 or 255, in the format's own type) restored as the 4th channel."""
    n = planar.shape[0]
    px = np.empty((n, 64, 4), dtype=planar.dtype)
    px[..., :3] = planar.transpose(0, 2, 1)
    px[..., 3] = alpha
    return px.reshape(n * 64, 4)


CHANNEL_BYTES = {0: 4, 1: 2, 2: 1}  # bh_out_format -> bytes per channel (RGBA32F, RGBA16F, BGRA8)


def rgbm_tile_bytes(fmt: int) -> int:
    """Bytes of one BH_LAYOUT_TILES_RGBM tile (include/bh_render.h): three planes of 64 channel values,
    then the 64-bit blackout mask word."""
    return 192 * CHANNEL_BYTES[fmt] + 8


def pack_rgbm_numpy(col: np.ndarray, zero: np.ndarray, k: int, S: int, stride: int, weights=None) -> np.ndarray:
    """Host mirror of the march kernel's BH_LAYOUT_TILES_RGBM store for shard k: `col` (H, W, 4) in the
    format's memory order (uint8 / float16 / float32 channels), `zero` (H, W) bool = the pixel's
    blackout_col is 0 (dot(col, col) < 1 in fp32).  Returns (stride, tile_bytes) uint8; pixels outside
    the frame are 0 and their mask bits clear."""
    H, W, _ = col.shape
    cb = col.dtype.itemsize
    out = np.zeros((stride, 192 * cb + 8), np.uint8)
    lane = np.arange(64)
    for t, (tx, ty) in enumerate(shard_tiles(W, H, k, S, weights)):
        px, py = tx * TILE + (lane & 7), ty * TILE + (lane >> 3)
        ok = (px < W) & (py < H)
        planes = np.zeros((3, 64), col.dtype)
        planes[:, ok] = col[py[ok], px[ok], :3].T
        out[t, :192 * cb] = planes.view(np.uint8).ravel()
        zt = np.zeros(64, bool)
        zt[ok] = zero[py[ok], px[ok]]
        m = sum(1 << int(i) for i in lane[zt])
        out[t, 192 * cb:] = np.frombuffer(np.uint64(m).tobytes(), np.uint8)
    return out


def unpack_rgbm_numpy(packed: np.ndarray, width: int, height: int, S: int, stride: int, dtype, alpha, weights=None):
    """Host mirror of bh_tiles_unpack_rgbm: gathered (S * stride, tile_bytes) uint8 -> (col, blackout),
    each (height, width, 4) of `dtype` with the constant `alpha` restored; blackout = col with the
    masked pixels' RGB zeroed."""
    cb = np.dtype(dtype).itemsize
    col = np.zeros((height, width, 4), dtype)
    bo = np.zeros((height, width, 4), dtype)
    lane = np.arange(64)
    for k in range(S):
        for t, (tx, ty) in enumerate(shard_tiles(width, height, k, S, weights)):
            tile = packed[k * stride + t]
            planes = tile[:192 * cb].view(dtype).reshape(3, 64)
            m = tile[192 * cb:].view(np.uint64)[0]
            zero = ((m >> lane.astype(np.uint64)) & np.uint64(1)).astype(bool)
            px, py = tx * TILE + (lane & 7), ty * TILE + (lane >> 3)
            ok = (px < width) & (py < height)
            col[py[ok], px[ok], :3] = planes[:, ok].T
            col[py[ok], px[ok], 3] = alpha
            keep = ok & ~zero
            bo[py[keep], px[keep], :3] = planes[:, keep].T
            bo[py[ok], px[ok], 3] = alpha
    return col, bo


RGBM14_TILE_BYTES = 344  # BH_LAYOUT_TILES_RGBM14 (include/bh_render.h): RGBA16F in 14-bit channels


def pack_rgbm14_numpy(col: np.ndarray, zero: np.ndarray, k: int, S: int, stride: int, weights=None) -> np.ndarray:
    """Host mirror of the march kernel's BH_LAYOUT_TILES_RGBM14 store (store_rgbm14) for shard k: `col`
    (H, W, 4) float16 whose RGB are in [0, 1] (fp16 bits < 0x4000), `zero` (H, W) bool as pack_rgbm_numpy.
    Per tile: 64 words r | g << 14 | (b & 0xF) << 28, 64 bytes (b >> 4) & 0xFF, b's bit-12 and bit-13
    ballot words, the mask word.  Returns (stride, 344) uint8; pixels outside the frame are 0."""
    H, W, _ = col.shape
    bits = col.view(np.uint16).astype(np.uint32)
    if (bits[..., :3] >= 0x4000).any():
        raise ValueError("RGBM14 carries fp16 channels in [0, 1] only")
    out = np.zeros((stride, RGBM14_TILE_BYTES), np.uint8)
    lane = np.arange(64)
    for t, (tx, ty) in enumerate(shard_tiles(W, H, k, S, weights)):
        px, py = tx * TILE + (lane & 7), ty * TILE + (lane >> 3)
        ok = (px < W) & (py < H)
        r, g, b = (np.zeros(64, np.uint32) for _ in range(3))
        r[ok], g[ok], b[ok] = bits[py[ok], px[ok], 0], bits[py[ok], px[ok], 1], bits[py[ok], px[ok], 2]
        zt = np.zeros(64, bool)
        zt[ok] = zero[py[ok], px[ok]]
        words = (r | (g << 14) | ((b & 0xF) << 28)).astype(np.uint32)
        hi = ((b >> 4) & 0xFF).astype(np.uint8)
        ballot = [sum(1 << int(i) for i in lane[m]) for m in (((b >> 12) & 1) == 1, ((b >> 13) & 1) == 1, zt)]
        out[t, :256] = words.view(np.uint8)
        out[t, 256:320] = hi
        out[t, 320:] = np.array(ballot, np.uint64).view(np.uint8)
    return out


def unpack_rgbm14_numpy(packed: np.ndarray, width: int, height: int, S: int, stride: int, weights=None):
    """Host mirror of bh_tiles_unpack_rgbm with BH_UNPACK_RGBM14: gathered (S * stride, 344) uint8 ->
    (col, blackout) float16 (height, width, 4), alpha 1.0 restored, blackout = col with the masked RGB 0."""
    col = np.zeros((height, width, 4), np.float16)
    bo = np.zeros((height, width, 4), np.float16)
    lane = np.arange(64)
    one = np.float16(1.0)
    for k in range(S):
        for t, (tx, ty) in enumerate(shard_tiles(width, height, k, S, weights)):
            tile = packed[k * stride + t]
            w = tile[:256].view(np.uint32).astype(np.uint64)
            hi = tile[256:320].astype(np.uint64)
            m12, m13, mz = (tile[320 + 8 * j:328 + 8 * j].view(np.uint64)[0] for j in range(3))
            sh = lane.astype(np.uint64)
            b = (w >> np.uint64(28)) | (hi << np.uint64(4)) | (((m12 >> sh) & np.uint64(1)) << np.uint64(12)) \
                | (((m13 >> sh) & np.uint64(1)) << np.uint64(13))
            rgb = np.stack([w & np.uint64(0x3FFF), (w >> np.uint64(14)) & np.uint64(0x3FFF), b], -1)
            rgb = rgb.astype(np.uint16).view(np.float16)
            zero = ((mz >> sh) & np.uint64(1)).astype(bool)
            px, py = tx * TILE + (lane & 7), ty * TILE + (lane >> 3)
            ok = (px < width) & (py < height)
            col[py[ok], px[ok], :3] = rgb[ok]
            col[py[ok], px[ok], 3] = one
            keep = ok & ~zero
            bo[py[keep], px[keep], :3] = rgb[keep]
            bo[py[ok], px[ok], 3] = one
    return col, bo


def gather_packed(packed, rank: int, world: int, gathered=None, group=None):
    """Gather every rank's packed tile buffer (same shape on all ranks) to rank 0.

    One torch.distributed.gather: RCCL on GPUs (rank 0 receives the 7 peers over 7 xGMI links at
    once), gloo in CPU tests.  Returns the list of buffers on rank 0, None elsewhere."""
    import torch.distributed as dist
    if world == 1:
        return [packed]
    if rank == 0 and gathered is None:
        import torch
        gathered = [torch.empty_like(packed) for _ in range(world)]
    dist.gather(packed, gathered if rank == 0 else None, dst=0, group=group)
    return gathered if rank == 0 else None


class GatherPipeline:
    """Frame pipeline over ranks: frame i is rendered into packed buffer i % depth, its gather to
    rank 0 is issued asynchronously right after (torch.distributed enqueues the collective on its
    own stream behind the render), so it runs over xGMI while frame i+1 renders; rank 0 then unpacks
    frame i.  Before frame i + depth reuses a buffer, the gather that read it is waited on (on the
    compute stream, not the host, for RCCL).  Rank 0 receives straight into one contiguous
    (world, stride*64, C) buffer per slot, so the unpack reads it without a concatenation.

        pipe = GatherPipeline(lambda: torch.empty(...), rank, world, on_frame)
        for i in range(K):
            render_into(pipe.buffer(i)); pipe.submit(i)
        pipe.drain()

    `on_frame(i, gathered)` runs on rank 0 once frame i's gather is complete (stream-ordered):
    `gathered` is the (world * stride * 64, C) buffer of all ranks' packed tiles.  With
    `side_stream` (rank 0, CUDA), on_frame is issued on that stream -- the unpack (HBM-bound) then
    overlaps the next frame's render (VALU-bound) instead of queueing behind it on the render
    stream; before a receive buffer is gathered into again, the render stream waits for the unpack
    that read it (and RCCL's stream follows the render stream).  `collective`: gather through
    torch.distributed even at world size 1 (default: only when world > 1; a one-rank group checks
    the collective calls on a 1-GPU box).

    `timing` (CUDA): HIP events per frame for the bench's per-rank breakdown (timeline()): `submitted`
    on the producer stream when the gather is issued (the end of the render), `gathered` when the
    frame's collective is complete as seen by rank 0's side stream (every rank's shard received), or by
    another rank's producer stream (its send buffer released), `unpacked` after rank 0's on_frame."""

    def __init__(self, make_buffer, rank: int, world: int, on_frame=None, depth: int = 2, group=None,
                 side_stream=None, collective=None, timing=False):
        import torch
        if depth < 1:
            raise ValueError("depth >= 1")
        self.rank, self.world, self.depth, self.group = rank, world, depth, group
        self.on_frame = on_frame
        self.bufs = [make_buffer() for _ in range(depth)]
        self.recv = None
        if rank == 0:
            b = self.bufs[0]
            self.recv = [torch.empty((world * b.shape[0], *b.shape[1:]), dtype=b.dtype, device=b.device)
                         for _ in range(depth)]
        self.pending = []  # (frame, work) in submission order
        self.side = side_stream if rank == 0 else None
        self.consumed = [None] * depth  # per slot: event after the on_frame that read recv[slot]
        self.collective = world > 1 if collective is None else bool(collective)
        self.timing = bool(timing)
        self.events = {}  # frame -> {"submitted" | "gathered" | "unpacked": torch.cuda.Event}

    def _mark(self, i: int, what: str, stream=None) -> None:
        if self.timing:
            import torch
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(stream if stream is not None else torch.cuda.current_stream())
            self.events.setdefault(i, {})[what] = ev

    def timeline(self, frames) -> dict:
        """Per-frame ms between the timing events of `frames` (synchronise first): gather = submitted ->
        gathered, unpack = gathered -> unpacked (rank 0 with a side stream)."""
        out = {"gather_ms": [], "unpack_ms": []}
        for i in frames:
            e = self.events.get(i, {})
            if "submitted" in e and "gathered" in e:
                out["gather_ms"].append(e["submitted"].elapsed_time(e["gathered"]))
            if "gathered" in e and "unpacked" in e:
                out["unpack_ms"].append(e["gathered"].elapsed_time(e["unpacked"]))
        return out

    def buffer(self, i: int):
        return self.bufs[i % self.depth]

    def submit(self, i: int) -> None:
        import torch.distributed as dist
        slot = i % self.depth
        if self.consumed[slot] is not None:  # the unpack that last read recv[slot] (side stream)
            import torch
            torch.cuda.current_stream().wait_event(self.consumed[slot])
            self.consumed[slot] = None
        self._mark(i, "submitted")
        if not self.collective:
            work = None
            if self.rank == 0:
                self.recv[slot].copy_(self.bufs[slot])
        else:
            gl = list(self.recv[slot].view(self.world, *self.bufs[slot].shape).unbind(0)) if self.rank == 0 else None
            work = dist.gather(self.bufs[slot], gl, dst=0, group=self.group, async_op=True)
        self.pending.append((i, work))
        while len(self.pending) >= self.depth:  # the next frame's buffer must be free
            self._finish_one()

    def _finish_one(self) -> None:
        i, work = self.pending.pop(0)
        slot = i % self.depth
        if work is not None:
            work.wait()  # the current stream: the send buffer may be rendered into again
        if self.side is None:
            self._mark(i, "gathered")
        if self.rank == 0 and self.on_frame is not None:
            if self.side is None:
                self.on_frame(i, self.recv[slot])
            else:
                import torch
                producer = torch.cuda.current_stream()
                with torch.cuda.stream(self.side):
                    if work is not None:
                        work.wait()  # the side stream: the received frame is complete
                    else:
                        self.side.wait_stream(producer)  # the local copy into recv[slot]
                    self._mark(i, "gathered", self.side)
                    self.on_frame(i, self.recv[slot])
                    self._mark(i, "unpacked", self.side)
                    ev = torch.cuda.Event()
                    ev.record(self.side)
                    self.consumed[slot] = ev

    def drain(self) -> None:
        while self.pending:
            self._finish_one()


def weak_scaling_frame(world: int, base_w: int = 4096, base_h: int = 2048) -> tuple[int, int]:
    """Frame for `world` GPUs with about base_w*base_h pixels per GPU at the base aspect (weak scaling)."""
    if world == 1:
        return base_w, base_h
    w = int(round(base_w * np.sqrt(world) / TILE)) * TILE
    return w, int(round(w * base_h / base_w / TILE)) * TILE
