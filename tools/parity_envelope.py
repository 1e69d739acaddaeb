"""Parity envelope (VERDICT r01 "Next round" 8; CPU only): how far a real WGSL implementation could
land from the normative oracle that every parity test pins the kernel to.  WGSL leaves pow / atan2
precision and the texture unit's filtering to the implementation; the oracle fixes one exact choice
for each.  Each variant swaps one choice (oracle/bh_oracle.c BHO_V_*):
  pow      pow(x, e) = exp2(e * log2(x)) in f32 (the usual GPU lowering), in rd_derivative and g/b^1.5
  tex8     bilinear weights with 8 fractional bits (texture units' sub-texel precision)
  nearest  LOD 0 treated as minification, so the sampler's min_filter Nearest (src/texture.rs:66-67)
  atan2f   atan2 in f32
and the frame is compared with the normative one: fate / n_rk mismatches, |delta| on matched pixels
(RGB, fp32), the share of pixels over the north-star 1e-4.

    python tools/parity_envelope.py [--width 1024 --height 512] > profiles/r02/parity_envelope.json"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--height", type=int, default=512)
    a = ap.parse_args()
    import black_hole_ray_marching_amd as bh
    import oracle
    from tests._cases import camera_uniform, uniforms
    sky = bh.synthetic_sky()
    W, H = a.width, a.height
    variants = {"pow": oracle.V_POW_EXP2LOG2, "tex8": oracle.V_TEX_8BIT, "nearest": oracle.V_TEX_NEAREST,
                "atan2f": oracle.V_ATAN2F, "pow+tex8+atan2f": oracle.V_POW_EXP2LOG2 | oracle.V_TEX_8BIT | oracle.V_ATAN2F}
    out = {"frame": f"{W}x{H}", "sky": "synthetic 4096x2048", "cases": []}
    for cam, cap in (("A", 512), ("B", 512), ("C", 1000), ("D", 512), ("E", 512)):
        cu, U = camera_uniform(cam, W, H), uniforms()
        ref = oracle.render_rows(cu.to_bytes(), bytes(U.to_c()), sky, W, H, cap, 3)
        for name, v in variants.items():
            got = oracle.render_rows(cu.to_bytes(), bytes(U.to_c()), sky, W, H, cap, 3, variant=v)
            match = (got[2] == ref[2]) & (got[3] == ref[3])
            d = np.abs(got[0][..., :3] - ref[0][..., :3]).max(axis=-1)
            dm = d[match]
            out["cases"].append({
                "camera": cam, "cap": cap, "variant": name,
                "fate_nrk_mismatch": round(float(1 - match.mean()), 6),
                "max_abs_delta_matched": float(dm.max()) if dm.size else 0.0,
                "p99_9_abs_delta_matched": float(np.quantile(dm, 0.999)) if dm.size else 0.0,
                "share_over_1e-4": round(float((d > 1e-4).mean()), 6),
                "bit_identical_share": round(float((d == 0).mean()), 6)})
            print(json.dumps(out["cases"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
