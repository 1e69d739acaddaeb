"""Count guarded-fallback (IEEE) steps of the exact kernel, and the wave-steps that skipped the SDF roots
(sdf_skip): BH_LIB=tools/variants/diag.so python tools/diag_slow.py  (diag.so: -DBH_DIAG_SLOW)"""
import ctypes as C
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch
import black_hole_ray_marching_amd as bh

lib = bh.load()
lib.bh_diag_slow_counts.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
lib.bh_diag_skip_counts.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
lib.bh_diag_far_count.argtypes = [C.POINTER(C.c_uint32)]
sky = bh.synthetic_sky()
from bench import CAMERAS  # noqa: E402

for cam, cap in (("A", 512), ("B", 512), ("C", 1000)):
    sc = bh.Scene(4096, 2048, sky=sky, max_iters=cap, math=bh.BH_MATH_EXACT)
    if cam != "A":
        sc.update(bh.Camera.look_at(*CAMERAS[cam], 4096, 2048))
    col = torch.empty((2048, 4096, 4), dtype=torch.float16, device="cuda")
    nrk = torch.empty((2048, 4096), dtype=torch.int16, device="cuda")
    a, b = C.c_uint32(), C.c_uint32()
    k, w, fw = C.c_uint32(), C.c_uint32(), C.c_uint32()
    lib.bh_diag_slow_counts(C.byref(a), C.byref(b))
    lib.bh_diag_skip_counts(C.byref(k), C.byref(w))
    lib.bh_diag_far_count(C.byref(fw))
    sc.render(col, None, fmt=bh.BH_OUT_RGBA16F, dbg_n_rk=nrk, schedule=bh.BH_SCHED_TILE)
    torch.cuda.synchronize()
    lib.bh_diag_slow_counts(C.byref(a), C.byref(b))
    lib.bh_diag_skip_counts(C.byref(k), C.byref(w))
    lib.bh_diag_far_count(C.byref(fw))
    steps = int(nrk.cpu().numpy().view("uint16").astype("int64").sum())
    print(f"camera {cam} cap {cap}: lane-steps total {steps}, slow lane-steps {a.value}, slow wave-steps {b.value}, "
          f"waves {4096*2048//64}; wave-steps {w.value}, root-free {k.value} ({k.value / max(w.value, 1):.3f}), far field {fw.value} ({fw.value / max(w.value, 1):.3f})")
