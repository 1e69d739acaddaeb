"""Post-processing chain (bh_bloom) on one GPU: time per frame of the Kawase
bloom + remix over a 4096x2048 BGRA8 frame (the march kernel's own two targets), HIP events on the
stream, fused (AUTO) and literal schedules.  `roofline` (tools/bloom_roofline.py): the chain's
algorithmic bytes (read col + blackout, write the surface: 12 B/pixel) against HBM, the reference's arithmetic
in flop-equivalents as a rate against the FP32 VALU peak (an op count, not executed instructions), and -- when
a committed rocprofv3 PMC summary of this frame size exists (profiles/r*/bloom_roof/roofline<W>.json, the newest) --
the hardware's executed VALU-issue, LDS and HBM busy fractions, time-weighted over the fused chain's kernels: as
`hardware` when the summary's library_sha256 is the loaded library's, else as `profiled_build_hardware` (another
build's counters, kept apart from this run's time).
    python tools/bench_bloom.py [--width 4096 --height 2048 --levels 3 --steps 100]"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import black_hole_ray_marching_amd as bh  # noqa: E402
from tools.bloom_roofline import chain_roofline  # noqa: E402

ROOT = Path(__file__).resolve().parent.parent


def hardware_busy(W, H):
    """Time-weighted VALU / LDS busy and HBM fraction of the fused chain's kernels from the newest committed PMC
    summary of this frame size, with the build it profiled (library_sha256; absent in round 5's summaries):
    (key, fields), key 'hardware' when that build is the loaded library, else 'profiled_build_hardware'."""
    from tools.bloom_roofline import library_sha256
    cands = sorted((ROOT / "profiles").glob(f"r*/bloom_roof/roofline{W}.json"))
    if not cands:
        return None
    f = cands[-1]
    d = json.loads(f.read_text())
    if d.get("height") != H or "kernels" not in d:
        return None
    t = sum(k["us"] * k["launches_per_chain"] for k in d["kernels"])
    out = {"source": str(f.relative_to(ROOT)), "kernel_us_per_chain": round(t, 2),
           "profiled_library_sha256": d.get("library_sha256"), "loaded_library_sha256": library_sha256()}
    for key in ("valu_busy", "lds_busy", "hbm_frac"):
        out[key] = round(sum(k.get(key, 0.0) * k["us"] * k["launches_per_chain"] for k in d["kernels"]) / t, 3)
    return out

p = argparse.ArgumentParser()
p.add_argument("--width", type=int, default=4096)
p.add_argument("--height", type=int, default=2048)
p.add_argument("--levels", type=int, default=3)
p.add_argument("--steps", type=int, default=100)
p.add_argument("--warmup", type=int, default=10)
p.add_argument("--schedule", choices=["both", "auto", "literal"], default="both")
args = p.parse_args()
W, H = args.width, args.height
scene = bh.Scene(W, H, sky=bh.synthetic_sky(), max_iters=512, math=bh.BH_MATH_EXACT)
col = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
bo = torch.empty_like(col)
out = torch.empty_like(col)
scene.render(col, bo, fmt=bh.BH_OUT_BGRA8_SRGB)
stream = torch.cuda.current_stream()
for name, sched in (("auto", bh.BH_BLOOM_AUTO), ("literal", bh.BH_BLOOM_LITERAL)):
    if args.schedule not in ("both", name):
        continue
    for _ in range(args.warmup):
        scene.bloom(col, bo, out, levels=args.levels, schedule=sched, stream=stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for a, b in ev:
        a.record(stream)
        scene.bloom(col, bo, out, levels=args.levels, schedule=sched, stream=stream)
        b.record(stream)
    torch.cuda.synchronize()
    ms = np.array([a.elapsed_time(b) for a, b in ev])
    alg = W * H * 12
    line = {"bloom_schedule": name, "width": W, "height": H, "levels": args.levels,
            "avg_ms": round(float(ms.mean()), 5), "min_ms": round(float(ms.min()), 5),
            "mpix_per_s": round(W * H / (ms.mean() / 1e3) / 1e6, 1),
            "roofline_hbm": {"bound": "hbm", "achieved": round(alg / (ms.mean() / 1e3) / 1e9, 1),
                             "peak": 8000.0, "unit": "GB/s",
                             "frac": round(alg / (ms.mean() / 1e3) / 1e9 / 8000.0, 4),
                             "algorithmic_bytes": alg,
                             "note": "read col + blackout, write the surface (BGRA8)"}}
    if name == "auto":
        line["roofline"] = chain_roofline(W, H, args.levels, float(ms.mean()))
        hw = hardware_busy(W, H)
        if hw:
            # only the build that was profiled may report its counters as this run's
            same = hw["profiled_library_sha256"] == hw["loaded_library_sha256"]
            line["roofline"]["hardware" if same else "profiled_build_hardware"] = hw
    print(json.dumps(line))
