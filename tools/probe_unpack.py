import sys, json, torch
sys.path.insert(0, ".")
import black_hole_ray_marching_amd as bh
from black_hole_ray_marching_amd import multigpu
dev = torch.device("cuda:0")
def t(fn, it=30):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(it)]
    for a, b in ev:
        a.record(); fn(); b.record()
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / it
for mb in (128, 256, 512, 1024):
    x = torch.empty(mb << 20, dtype=torch.uint8, device=dev); y = torch.empty_like(x)
    ms = t(lambda: y.copy_(x))
    print(json.dumps({"copy_MiB": mb, "ms": round(ms, 4), "GBps": round(2 * x.numel() / ms / 1e6, 1)}))
    del x, y
W, H = 11584, 5792
frame = torch.empty((H, W, 4), dtype=torch.float16, device=dev)
for S in (1, 2, 4, 8):
    stride = multigpu.packed_stride(W, H, S)
    packed = torch.zeros((S * stride, 3, 64), dtype=torch.float16, device=dev)
    ms = t(lambda: bh.tiles_unpack_rgb(packed, frame, W, H, S, stride, bh.BH_OUT_RGBA16F))
    nb = packed.numel() * 2 + frame.numel() * 2
    print(json.dumps({"S": S, "ms": round(ms, 4), "GBps": round(nb / ms / 1e6, 1)}))
    del packed
