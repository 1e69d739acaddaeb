"""Shader clock and HBM load latency after each frame (tools/ubench/clock_probe.so, one wave reading s_memtime against the
100 MHz s_memrealtime) beside the frame's kernel time: tells the clock ramp from the cost order's
learning in the first frames after an idle GPU (VERDICT r01 "Next round" 6).  Series: learned and
static order after a 1 s idle, then learned right after 200 busy frames.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/ubench/clock_probe.hip -o tools/ubench/clock_probe.so
    python tools/clock_series.py [--frames 60]"""
import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=60)
    p.add_argument("--spin", type=int, default=20000)
    p.add_argument("--chase", type=int, default=200, help="dependent HBM loads per latency probe")
    a = p.parse_args()
    import torch
    import black_hole_ray_marching_amd as bh
    lib = C.CDLL(str(ROOT / "tools" / "ubench" / "clock_probe.so"))
    lib.clock_probe.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    lib.chase_probe.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    lib.chip_clock_probe.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    B = 1024  # one-wave workgroups of the whole-chip probe (4 per CU, all resident at once)
    N = 1 << 28  # 1 GiB chain: p -> (p + a ~4 MiB prime stride) mod N, every load a new line and page
    chain = ((torch.arange(N, dtype=torch.int64, device="cuda") + 1048573) % N).to(torch.int32)
    sky = bh.synthetic_sky()
    col = torch.empty((2048, 4096, 4), dtype=torch.float16, device="cuda")
    bo = torch.empty_like(col)
    st = torch.cuda.current_stream()
    out = {}

    def series(name, flag, frames):
        scene = bh.Scene(4096, 2048, sky=sky, max_iters=512, math=bh.BH_MATH_EXACT)
        probe = torch.zeros((frames, 4), dtype=torch.int64, device="cuda")
        lat = torch.zeros((frames, 2), dtype=torch.int64, device="cuda")
        chip = torch.zeros((frames, B, 4), dtype=torch.int64, device="cuda")
        cev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(frames)]
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(frames)]
        for i, (s, e) in enumerate(ev):
            s.record()
            scene.render(col, bo, fmt=bh.BH_OUT_RGBA16F, schedule=bh.BH_SCHED_TILE | flag)
            e.record()
            if lib.clock_probe(C.c_void_p(probe[i].data_ptr()), a.spin, C.c_void_p(st.cuda_stream)) != 0:
                raise SystemExit("clock_probe launch failed")
            if lib.chase_probe(C.c_void_p(chain.data_ptr()), C.c_void_p(lat[i].data_ptr()), a.chase,
                               C.c_void_p(st.cuda_stream)) != 0:
                raise SystemExit("chase_probe launch failed")
            cev[i][0].record()
            if lib.chip_clock_probe(C.c_void_p(chip[i].data_ptr()), B, a.spin, C.c_void_p(st.cuda_stream)) != 0:
                raise SystemExit("chip_clock_probe launch failed")
            cev[i][1].record()
        torch.cuda.synchronize()
        scene.close()
        pr = probe.cpu().numpy()
        mhz = [round(100.0 * int(c) / int(r), 1) if r else None for c, r in pr[:, :2]]
        if name:
            out[name] = {"ms": [round(s.elapsed_time(e), 4) for s, e in ev], "shader_mhz": mhz,
                         "hbm_load_ns": [round(int(t) * 10.0 / a.chase, 1) for t in lat.cpu().numpy()[:, 0]],
                         "chip_probe_ms": [round(s.elapsed_time(e), 4) for s, e in cev],
                         "xcd_mhz": xcd_mhz(chip.cpu().numpy())}

    def xcd_mhz(c):  # (frames, B, 4) -> per frame, per XCD: mean shader MHz of its workgroups
        res = []
        for f in c:
            d = {}
            for dm, dr, x, _ in f:
                if dr:
                    d.setdefault(int(x), []).append(100.0 * int(dm) / int(dr))
            res.append([round(sum(v) / len(v)) for _, v in sorted(d.items())])
        return res

    time.sleep(1.0)
    series("learned_after_idle", 0, a.frames)
    time.sleep(1.0)
    series("static_after_idle", bh.BH_SCHED_FLAG_STATIC_ORDER, a.frames)
    series(None, 0, 200)
    series("learned_hot", 0, a.frames)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
