"""Shader clock under a frame-like VALU load (tools/ubench/clock_probe.so heavy_clock_probe: 8 waves per
SIMD of independent FMA chains), launched back to back after a 1 s idle: kernel time (HIP events) and the
per-XCD shader clock each launch ran at (s_memtime / s_memrealtime).  Tells whether the slow first ~40
frames after an idle GPU (profiles/r02b/ramp.log) are the clock under load.

    python tools/heavy_clock.py [--launches 60] [--spin 4000]"""
import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--launches", type=int, default=60)
    p.add_argument("--spin", type=int, default=4000)
    a = p.parse_args()
    import torch
    lib = C.CDLL(str(ROOT / "tools" / "ubench" / "clock_probe.so"))
    lib.heavy_clock_probe.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    B = 8 * cus
    out = torch.zeros((a.launches, B, 4), dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream()
    lib.heavy_clock_probe(C.c_void_p(out[0].data_ptr()), B, 100, C.c_void_p(st.cuda_stream))
    torch.cuda.synchronize()
    time.sleep(1.0)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.launches)]
    for i, (s, e) in enumerate(ev):
        s.record()
        if lib.heavy_clock_probe(C.c_void_p(out[i].data_ptr()), B, a.spin, C.c_void_p(st.cuda_stream)) != 0:
            raise SystemExit("heavy_clock_probe launch failed")
        e.record()
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    res = {"blocks": B, "ms": [], "mhz_min": [], "mhz_mean": []}
    for i, (s, e) in enumerate(ev):
        mhz = 100.0 * o[i, :, 0] / o[i, :, 1]
        res["ms"].append(round(s.elapsed_time(e), 4))
        res["mhz_min"].append(round(float(mhz.min())))
        res["mhz_mean"].append(round(float(mhz.mean())))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
