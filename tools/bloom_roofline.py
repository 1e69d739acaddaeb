"""Roofline of the bloom chain (bh_bloom: Kawase bloom + remix), per chain and per kernel.

Algorithmic work (what the reference computes; src/bloom.rs:53-71, the WGSL passes it runs): the chain of
the literal schedule -- the reference's own render passes, listed by bh_bloom_check -- counted per output
pixel in flop-equivalents, every f32 operation and every texel decode (the sRGB / alpha table lookup the
texture unit does) and every channel encode (the Bgra8UnormSrgb store) counted 1:
  bilinear sample (textureSample, 4 channels)      16 decodes + 4 x 9 lerp ops (6 mul, 3 add)       =  52
  kawase_upsample.wgsl:29-39  8 samples, sum with weights 1/2, / 12: 8 x 52 + 4 x (7 add + 4 x2 + 1 div)
                              + 4 encodes                                                            = 468
  kawase_downsample.wgsl (returns its centre tap) / copy.wgsl: 1 sample + 4 encodes                 =  56
  remix.wgsl:22-25            2 samples + 4 x (mul, add) + 4 encodes                                  = 116
Algorithmic HBM bytes: read col + blackout, write the surface (BGRA8): 12 B per pixel.  Peaks: FP32 VALU
78.6 T lane-ops/s (1024 SIMDs x 32 lanes x 2.4 GHz, no FMA: the filters' products and sums round one by one),
HBM 8 TB/s, LDS 157 TB/s (256 B/clk/CU x 256 CUs x 2.4 GHz, ds_read_b128; MI355X_MICROARCH.md §LDS).

With a rocprofv3 directory (tools/gpu/bloom_roofline.sh: kernel trace + PMC passes of tools/bench_bloom.py),
every kernel of the fused chain gets its measured time, its executed VALU and LDS instructions per output
pixel (lane slots: instructions x 64 / pixels), VALU-issue busy (2 cycles per wave64 VALU op on a SIMD-32),
LDS-array busy (SQ_LDS_IDX_ACTIVE over CU cycles), bank-conflict share and HBM bytes (FETCH_SIZE x2 +
WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md) against the peaks.

    python tools/bloom_roofline.py --width 1920 --height 1080 [--pmc DIR] [--chain-ms 0.129]
"""
import argparse
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

SAMPLE = 16 + 4 * 9
OPS = {"up": 8 * SAMPLE + 4 * 12 + 4, "down": SAMPLE + 4, "copy": SAMPLE + 4, "remix": 2 * SAMPLE + 8 + 4}
PEAK_VALU = 78.6e12      # FP32 lane-ops / s, no FMA
PEAK_HBM = 8.0e12        # B / s
PEAK_LDS = 157.3e12      # B / s (256 B/clk/CU)
CLOCK_HZ = 2.4e9
CUS, SIMDS = 256, 1024


FUSED_WORK = {  # bh_bloom_check form of the fused chain -> the reference passes its output pixels carry
    "sepq": None, "sep": None, "yq12": ("up", "remix"), "yq0": ("up", "remix"), "y1": ("up", "remix"),
    "final48": ("up", "remix", "remix"), "final0": ("up", "remix", "remix"), "final": ("up", "remix", "remix"),
    "up2_12": ("up",), "up2_3": ("up",), "up2_0": ("up",), "pass_up": ("up",), "pass_up_tap": ("up",),
    "pass_down": ("down",), "pass_copy": ("copy",), "pass_remix": ("remix",), "remix_plan": ("remix",),
    "remix2_plan": ("remix", "remix"), "fixup/1": (), "fixup/1r": (), "fixup/2": (), "fixup/2r": (),
    # the general chain's same-size copies where they are not identities (a copy pass or the blur's same-size down)
    "same_copy": ("copy",),
}


def minimal_ops(launches):
    """The reference's arithmetic of the passes the output actually depends on -- the fused chain's launches,
    each counted as the reference passes it computes (a separable pass with the EPI_Y epilogue: up + remix,
    EPI_FINAL: up + 2 remixes; down2: its two downsamples; the fix-ups recompute pixels counted already):
    the reference's own chain minus its identity copies and the repeated Y of its second loop iteration."""
    total = 0
    for form, ow, oh, tw, th, rx, ry in launches:
        if form.startswith("sep"):
            kinds = {"0": ("up",), "1": ("up", "remix"), "2": ("up", "remix", "remix")}[form.split("/")[1][0]]
        elif form in ("down2", "down2f"):  # down2f: fused into the Y launch before it
            total += OPS["down"] * rx * ry  # the intermediate level (mw x mh)
            kinds = ("down",)
        else:
            kinds = FUSED_WORK[form]
        total += sum(OPS[k] for k in kinds) * ow * oh
    return total


def reference_ops(W, H, levels):
    """The reference chain's work: the literal schedule's passes (its render passes one by one)."""
    import black_hole_ray_marching_amd as bh
    total, passes = 0, defaultdict(int)
    for form, ow, oh, *_ in bh.bloom_check(W, H, levels, bh.BH_BLOOM_LITERAL):
        kind = {"pass_up": "up", "pass_up_tap": "up", "pass_down": "down", "pass_copy": "copy",
                "pass_remix": "remix"}.get(form)
        if kind is None:
            if form.startswith("sep") or form.startswith("up2"):
                kind = "up"  # an up pass the launcher ran in its separable / 2:1 form
            else:
                raise SystemExit(f"unexpected literal-schedule form {form}")
        total += OPS[kind] * ow * oh
        passes[kind] += 1
    # the literal schedule copies the blackout input once with hipMemcpyAsync (copy_in[0] = X): no arithmetic
    return total, dict(passes)


# kernel name (rocprofv3) -> bh_bloom_check form of the fused chain
def form_of(name):
    n = name.split("(")[0]
    if "up_sepq_kernel<" in n:
        a = n.split("<")[1].rstrip(">").split(",")
        fix = "f" if len(a) > 4 and a[4].strip() == "true" else ""
        return f"sepq{int(a[0])}{'r' if a[2].strip() == 'true' else ''}/{int(a[1].strip().rstrip('u'))}{fix}"
    if "up_sep_kernel<" in n:
        a = n.split("<")[1].rstrip(">").split(",")
        return f"sep{int(a[0])}{'r' if a[2].strip() == 'true' else ''}/{int(a[1].strip().rstrip('u'))}"
    for k, f in (("same_copy_kernel", "same_copy"), ("fixup_gather_kernel<1u>", "fixup/1"), ("fixup_gather_kernel<2u>", "fixup/2"),
                 ("fixup_kernel<1u>", "fixup/1"), ("fixup_kernel<2u>", "fixup/2"), ("down2_kernel", "down2"),
                 ("bloom_yq_kernel<12>", "yq12"), ("bloom_yq_kernel<0>", "yq0"), ("bloom_yq_kernel<12, false>", "yq12"),
                 ("bloom_yq_kernel<0, false>", "yq0"), ("bloom_yq_kernel<12, true>", "yq12"),
                 ("bloom_yq_kernel<0, true>", "yq0"), ("bloom_y_kernel", "y1"),
                 ("bloom_final_kernel<48>", "final48"), ("bloom_final_kernel<0>", "final0"),
                 ("up2_kernel<12>", "up2_12"), ("up2_kernel<3>", "up2_3"), ("up2_kernel<0>", "up2_0"),
                 ("remix2_plan_kernel", "remix2_plan"), ("remix_plan_kernel", "remix_plan"),
                 ("pass_kernel<0u>", "pass_copy"), ("pass_kernel<1u>", "pass_down"), ("pass_kernel<2u>", "pass_up"),
                 ("pass_kernel<3u>", "pass_remix")):
        if k in n:
            return f
    return None


def launch_pixels(launches):
    """form -> output pixels per chain (a fix-up: its pixels; down2: the final level's)."""
    px = defaultdict(int)
    for form, ow, oh, tw, th, rx, ry in launches:
        if form.startswith("fixup"):
            px[form] += tw * oh + th * ow  # n_cols columns of H pixels + n_rows rows of W
        else:
            px[form] += ow * oh
    return px


def pmc(dirname):
    """Per kernel name: counters averaged per dispatch, and the trace's average duration (s)."""
    cnt = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{dirname}/p*/**/*counter_collection.csv", recursive=True):
        by = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            d = by[(r["Kernel_Name"], r["Dispatch_Id"])]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (k, _), cs in by.items():
            for c, v in cs.items():
                cnt[k][c].append(v)
    avg = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in cnt.items()}
    times = {}
    for f in glob.glob(f"{dirname}/trace/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            times[r["Name"]] = (float(r["AverageNs"]) * 1e-9, int(r["Calls"]))
    return avg, times


def chain_roofline(W, H, L, chain_ms, ref=None, mini=None):
    """The chain at `chain_ms` (bench_bloom's line) against the FP32 VALU and HBM peaks: 12 algorithmic B per
    pixel against HBM (a true fraction), and the reference's arithmetic in flop-equivalents -- the minimal
    dataflow's and the whole reference chain's (all 21 passes at levels 3) -- as a rate against the VALU peak.
    That rate is the reference's op count, not the executed instructions: the fused kernels share texel decodes
    between pixels (the 2:1 quad forms, the tile windows) and skip the sampler's coordinate work, so its ratio to
    the peak can exceed 1 (4096x2048).  The executed VALU fraction is the hardware summary's valu_busy
    (bench_bloom.hardware_busy, from rocprofv3 PMC)."""
    import black_hole_ray_marching_amd as bh
    if ref is None:
        ref, _ = reference_ops(W, H, L)
    if mini is None:
        mini = minimal_ops(bh.bloom_check(W, H, L, bh.BH_BLOOM_AUTO))
    t = chain_ms * 1e-3
    return {"bound": "latency (VALU, LDS and HBM all below their peaks; DESIGN.md §7b)",
            "reference_work": {"flop_eq_per_chain": mini, "rate_tops": round(mini / t / 1e12, 3),
                               "reference_op_rate_over_valu_peak": round(mini / t / PEAK_VALU, 4),
                               "reference_chain_flop_eq": ref,
                               "reference_chain_op_rate_over_valu_peak": round(ref / t / PEAK_VALU, 4),
                               "peak_tops": PEAK_VALU / 1e12,
                               "unit": "flop-eq (f32 op, texel decode, channel encode = 1 each)",
                               "note": "the reference's op count per chain time, not executed instructions (can "
                                       "exceed the peak); the executed fraction is hardware.valu_busy"},
            "hbm": {"achieved_gbs": round(12 * W * H / t / 1e9, 1), "peak_gbs": PEAK_HBM / 1e9,
                    "frac": round(12 * W * H / t / PEAK_HBM, 4), "algorithmic_bytes": 12 * W * H}}


def library_sha256() -> str:
    """sha256 (16 hex) of the libbh_render.so this process loads: ties a PMC summary to the build it profiled"""
    import hashlib
    from black_hole_ray_marching_amd import _abi
    return hashlib.sha256(_abi.LIB_PATH.read_bytes()).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--pmc", default="", help="rocprofv3 output directory (trace/ and p*/ passes)")
    ap.add_argument("--chain-ms", type=float, default=0.0, help="the chain's time (bench_bloom avg_ms)")
    a = ap.parse_args()
    import black_hole_ray_marching_amd as bh
    W, H, L = a.width, a.height, a.levels
    ref, passes = reference_ops(W, H, L)
    fused = bh.bloom_check(W, H, L, bh.BH_BLOOM_AUTO)
    mini = minimal_ops(fused)
    out = {"width": W, "height": H, "levels": L, "library_sha256": library_sha256(), "reference_passes": passes,
           "reference_flop_eq_per_chain": ref, "reference_flop_eq_per_pixel": round(ref / (W * H), 1),
           "minimal_flop_eq_per_chain": mini, "minimal_flop_eq_per_pixel": round(mini / (W * H), 1),
           "algorithmic_bytes": 12 * W * H, "fused_launches": [" ".join(map(str, x)) for x in fused]}
    if a.chain_ms:
        out["chain"] = chain_roofline(W, H, L, a.chain_ms, ref, mini)
    if a.pmc:
        avg, times = pmc(a.pmc)
        px = launch_pixels(fused)
        kern = []
        tot_t = 0.0
        for name, (t, calls) in sorted(times.items(), key=lambda x: -x[1][0] * x[1][1]):
            f = form_of(name)
            if f is None or f not in px:
                continue
            c = avg.get(name, {})
            n_launch = sum(1 for x in fused if x[0] == f)
            pix = px[f] / max(n_launch, 1)  # per dispatch
            row = {"kernel": name.split("(")[0].replace("bh::bloom::", "").replace("void ", ""), "form": f,
                   "us": round(t * 1e6, 2), "launches_per_chain": n_launch, "pixels": int(pix)}
            tot_t += t * n_launch
            if c.get("SQ_INSTS_VALU"):
                row["valu_per_px"] = round(c["SQ_INSTS_VALU"] * 64 / pix, 1)
                row["lds_instr_per_px"] = round(c.get("SQ_INSTS_LDS", 0) * 64 / pix, 2)
                cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8 or t * CLOCK_HZ
                row["valu_busy"] = round(c["SQ_INSTS_VALU"] * 2 / (cyc * SIMDS), 3)
                if c.get("SQ_LDS_IDX_ACTIVE"):
                    row["lds_busy"] = round(c["SQ_LDS_IDX_ACTIVE"] / (cyc * CUS), 3)
                    row["lds_bank_conflict_share"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 3)
                if c.get("SQ_WAVE_CYCLES"):
                    row["wait_share"] = round(c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"], 3)
            if c.get("FETCH_SIZE") is not None or c.get("WRITE_SIZE") is not None:
                hb = 2 * c.get("FETCH_SIZE", 0) * 1024 + c.get("WRITE_SIZE", 0) * 1024
                row["hbm_bytes"] = int(hb)
                row["hbm_frac"] = round(hb / t / PEAK_HBM, 4)
            kern.append(row)
        out["kernels"] = kern
        out["kernel_us_per_chain"] = round(tot_t * 1e6, 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
