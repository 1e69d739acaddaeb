// bh_march.hpp — the geodesic ray-march kernel for gfx950 (CDNA4), one lane per pixel.
//
// Included by exactly two translation units:
//   bh_march_exact.hip  (BH_FAST 0; built -ffp-contract=off, correctly-rounded f32 div/sqrt):
//       same op sequence as the normative arithmetic of oracle/bh_oracle.c -> bit-exact parity;
//   bh_march_fast.hip   (BH_FAST 1; built -ffp-contract=fast, hardware rcp/rsq/sqrt):
//       algebraically identical reformulation for throughput -> tolerance parity.
//
// Semantics follow src/black_hole_maybe.wgsl (reference): fs_main :360-370, get_col :259-345,
// get_delta_photon_rk4 :134-151, rd_derivative :125-127, sdf* :91-123.  Layout: each wave64 owns
// one 8x8 pixel tile (SIMD efficiency 0.72 vs 0.67 for 64x1 rows); RK state stays in
// VGPRs; the 256-entry sRGB decode table is staged in LDS once per workgroup; the 32 MiB RGBA8 sky
// is read with 4 dword gathers per escaped ray (L2/MALL-resident).
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include "bh_common.hpp"
#include "bh_crmath.hpp"
#include "bh_srgb.hpp"

#ifndef BH_FAST
#error "define BH_FAST to 0 or 1"
#endif
// (rd_derivative's reciprocal from the root's own v_rsq, crm::rcp_from_rsq, instead of a v_rcp of Q: four
// fewer transcendentals per RK step, but NOT exact -- 60 (numerator, Q) pairs, at Q significands next to
// 2 (e.g. n = 1, Q = 0x2cffffff), round the other way (selftest op 13) -- so the march keeps rcp_refined.)

namespace bh {
namespace BH_NS {

struct v3 { float x, y, z; };

__device__ __forceinline__ v3 mk(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 smul(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
// per-component select (an aggregate `c ? a : b` keeps the struct in scratch memory)
__device__ __forceinline__ v3 sel(bool c, v3 a, v3 b) { return mk(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }
__device__ __forceinline__ v3 cross(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

#if BH_FAST
__device__ __forceinline__ float rsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float fsqrt(float x) { return __builtin_sqrtf(x); }  // v_sqrt_f32 in this TU
__device__ __forceinline__ float len(v3 a) { return fsqrt(dot(a, a)); }
__device__ __forceinline__ v3 normalize(v3 a) { return muls(a, rsq(dot(a, a))); }
#else
__device__ __forceinline__ float len(v3 a) { return __builtin_sqrtf(dot(a, a)); }  // correctly rounded
__device__ __forceinline__ v3 divs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ v3 normalize(v3 a) { return divs(a, len(a)); }
// normative pow forms (oracle/bh_oracle.c header): three correctly rounded f32 ops each
__device__ __forceinline__ float pow25(float q) { return (q * q) * __builtin_sqrtf(q); }
__device__ __forceinline__ float pow15(float c) { return c * __builtin_sqrtf(c); }

// The per-ray set-up and shading ops on the cheap correctly rounded cores of bh_crmath.hpp (the same
// bits as the IEEE forms above, proofs at each).
//
// normalize(v) = v / sqrt(dot(v, v)): exact when q = dot(v, v) is in [2^-80, 2^120] (inside the sqrt
// core's domain, and then the length is in the division core's [2^-40, 2^60], which also bounds
// every |v_i| <= 2^60) and every component is 0 or >= 2^-60 in magnitude.  Otherwise the lanes
// concerned take the IEEE form (a wave-uniform branch; never seen on real frames).
__device__ __forceinline__ v3 normalize_x(v3 v) {
    const float q = dot(v, v);
    const float l = crm::sqrt_core(q);
    const crm::Rcp R = crm::rcp_refined(l);
    const v3 n = mk(crm::div_core(v.x, R), crm::div_core(v.y, R), crm::div_core(v.z, R));
    const bool bad = !(q >= 0x1p-80f && q <= 0x1p120f) |
                     (crm::kmin3(crm::key(v.x), crm::key(v.y), crm::key(v.z)) < crm::KEY_MIN);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(bad) != 0ull, 0)) {
        if (bad) return normalize(v);
    }
    return n;
}
// c * sqrt(c) for a bilinear sky sample c: c is +0 or in [2^-60, 1] (texels decode to 0 or
// >= 3.0e-4, the bilinear weights are 0 or >= 2^-24: two weight products keep c >= 1.8e-18), so
// the sqrt core is exact for every c > 0 and c = +0 gives +0 as c * sqrt(c) does.
__device__ __forceinline__ float pow15_x(float c) { return c > 0.0f ? c * crm::sqrt_core(c) : c; }
#endif

constexpr float MIN_DIST = 0.001f;        // :80
constexpr float TWO_PI = 6.28318530718f;  // :82
constexpr float ONE_PI = 3.14159265359f;  // :83

// sdf (:119-123) with the scene-flag selection of bh_render.h.
__device__ __forceinline__ float sdf(v3 p, float rs, uint32_t flags) {
    float d = __builtin_inff();
    if (flags & BH_SCENE_DISC) {
        // sdf_accretion_disk(p, 0, 6RS, 3RS) = max(max(rho - 6RS, -(rho - 3RS)), |p.y| - 0.02)
        float rho = __builtin_sqrtf(p.x * p.x + p.z * p.z);
        d = fmaxf(fmaxf(rho - 6.0f * rs, -(rho - 3.0f * rs)), fabsf(p.y - 0.0f) - 0.02f);
    }
    if (flags & BH_SCENE_MARKERS) {
#if BH_FAST
        // min of the four sphere SDFs == sqrt(min of squared distances) - 0.5 (sqrt is monotone);
        // spheres (0,+-10,-10), (+-10,0,-10) (:107-117)
        float ay = fabsf(p.y) - 10.0f, ax = fabsf(p.x) - 10.0f, dz = p.z + 10.0f;
        float q = fminf(p.x * p.x + ay * ay, ax * ax + p.y * p.y) + dz * dz;
        float m = __builtin_sqrtf(q) - 0.5f;
#else
        // sdf_sphere = length(centre - p) - r for the four spheres, each squared length evaluated
        // exactly as written ((dx*dx + dy*dy) + dz*dz with dx = cx - px, ...).  Shared terms are
        // computed once (identical roundings) and min(sqrt(qi) - 0.5) == sqrt(min(qi)) - 0.5
        // exactly, because correctly rounded sqrt and x - 0.5 are monotone: one sqrt, bit-exact.
        const float xx = p.x * p.x, yy = p.y * p.y;          // (0 - p)^2 == p^2
        const float dz = -10.0f - p.z, zz = dz * dz;
        const float a1 = 10.0f - p.y, a2 = -10.0f - p.y, b3 = 10.0f - p.x, b4 = -10.0f - p.x;
        const float q1 = (xx + a1 * a1) + zz, q2 = (xx + a2 * a2) + zz;
        const float q3 = (b3 * b3 + yy) + zz, q4 = (b4 * b4 + yy) + zz;
        float m = __builtin_sqrtf(fminf(q1, fminf(q2, fminf(q3, q4)))) - 0.5f;
#endif
        d = (flags & BH_SCENE_DISC) ? fminf(d, m) : m;
    }
    return d;
}

// rd_derivative (:125-127) = (s * ro) / pow(dot(ro,ro), 2.5), s = ((DP*RS)*-1.5)*h2 hoisted per ray.
__device__ __forceinline__ v3 accel(v3 p, float s) {
#if BH_FAST
    float iq = rsq(dot(p, p));
    float iq2 = iq * iq;
    float f = s * (iq2 * iq2 * iq);
    return muls(p, f);
#else
    float q = pow25(dot(p, p));
    return mk((s * p.x) / q, (s * p.y) / q, (s * p.z) / q);
#endif
}

struct Ray {
    v3 col;
    uint32_t n_rk;
    uint32_t fate;
};

// x, y clamped to the texture; 32-bit element index (bh_create: at most 2^30 texels), so the gather
// address is one 32-bit multiply-add and one 64-bit shift-add
__device__ __forceinline__ uint32_t texel_u32(const MarchArgs& a, int32_t x, int32_t y) {
    return a.sky[(uint32_t)y * a.sky_w + (uint32_t)x];
}
__device__ __forceinline__ v3 decode(const float* lut, uint32_t t) {
    return mk(lut[t & 0xffu], lut[(t >> 8) & 0xffu], lut[(t >> 16) & 0xffu]);
}
// lo <= hi: one v_med3_i32
__device__ __forceinline__ int32_t clampi(int32_t v, int32_t lo, int32_t hi) { return min(max(v, lo), hi); }

// textureSampleLevel(t_diffuse, s_diffuse, uv, 0) on Rgba8UnormSrgb, mag=Linear, clamp-to-edge
// (src/texture.rs:41,62-70): decode texels, then bilinear with fp32 weights.
__device__ __forceinline__ v3 sample_sky(const MarchArgs& a, const float* lut, float u, float v) {
    if (u != u || v != v) return decode(lut, texel_u32(a, 0, 0));  // Q8
    float tx = u * (float)a.sky_w - 0.5f;
    float ty = v * (float)a.sky_h - 0.5f;
    // fminf(fmaxf(t, -1), n) for the non-NaN t here: one v_med3_f32
    tx = __builtin_amdgcn_fmed3f(tx, -1.0f, (float)a.sky_w);
    ty = __builtin_amdgcn_fmed3f(ty, -1.0f, (float)a.sky_h);
    float fx0 = floorf(tx), fy0 = floorf(ty);
    float fa = tx - fx0, fb = ty - fy0;
    int32_t x0 = (int32_t)fx0, y0 = (int32_t)fy0;
    const int32_t wm = (int32_t)a.sky_w - 1, hm = (int32_t)a.sky_h - 1;
    int32_t x1 = clampi(x0 + 1, 0, wm), y1 = clampi(y0 + 1, 0, hm);
    x0 = clampi(x0, 0, wm);
    y0 = clampi(y0, 0, hm);
    // the four gathers first, then the decodes: one wait for all four (in the source-order build each
    // decode would otherwise wait for its own load)
    const uint32_t w00 = texel_u32(a, x0, y0), w10 = texel_u32(a, x1, y0);
    const uint32_t w01 = texel_u32(a, x0, y1), w11 = texel_u32(a, x1, y1);
    v3 t00 = decode(lut, w00), t10 = decode(lut, w10);
    v3 t01 = decode(lut, w01), t11 = decode(lut, w11);
    float ia = 1.0f - fa, ib = 1.0f - fb;
    v3 top = add(muls(t00, ia), muls(t10, fa));
    v3 bot = add(muls(t01, ia), muls(t11, fa));
    return add(muls(top, ib), muls(bot, fb));
}

// ---- per-ray pieces of get_col (:259-345) -------------------------------------------------------

// Per-frame invariants (identical for every pixel: ro0 == camera.pos, :363).
struct Frame {
    v3 ro0;
    v3 cps;      // photon-sphere centre -normalize(ro0) * 1.5 * RS  (:294)
    float k;     // (DP * RS) * -1.5: the scalar prefix of rd_derivative (:126)
};
__device__ __forceinline__ Frame make_frame(const MarchArgs& a) {
    Frame f;  // invariants precomputed on the host (bh_host.cpp, frame_constants)
    f.ro0 = mk(a.pos[0], a.pos[1], a.pos[2]);
    f.cps = mk(a.cps[0], a.cps[1], a.cps[2]);
    f.k = a.kfac;
    return f;
}

// vs_main + rasteriser interpolation + fs_main :362 for pixel (px, py): the world-space corner rays of
// the screen triangle (3,1),(-1,1),(-1,-3) interpolated at the pixel centre, normalised.
// Exact mode: the two divisions use the division core (numerators in [0.5, 2^32], denominators 2W,
// 2H in [2, 2^33]: always inside its domain) with the reciprocals RN(1/2W), RN(1/2H) from the host, and
// the normalisation normalize_x.
__device__ __forceinline__ v3 pixel_ray(const MarchArgs& a, uint32_t px, uint32_t py) {
#if BH_FAST
    const float l0 = ((float)px + 0.5f) / (2.0f * (float)a.width);
    const float l2 = ((float)py + 0.5f) / (2.0f * (float)a.height);
#else
    const float l0 = crm::div_core((float)px + 0.5f, crm::Rcp{2.0f * (float)a.width, a.rw2});
    const float l2 = crm::div_core((float)py + 0.5f, crm::Rcp{2.0f * (float)a.height, a.rh2});
#endif
    const float l1 = (1.0f - l0) - l2;
    const v3 d = add(add(smul(l0, mk(a.c0[0], a.c0[1], a.c0[2])), smul(l1, mk(a.c1[0], a.c1[1], a.c1[2]))),
                     smul(l2, mk(a.c2[0], a.c2[1], a.c2[2])));
#if BH_FAST
    return normalize(d);
#else
    return normalize_x(d);
#endif
}

// s = ((DP*RS)*-1.5) * h2 with h2 = |ro0 x rd0|^2 (:262-263), hoisted out of rd_derivative.
__device__ __forceinline__ float ray_s(const Frame& f, v3 rd0) {
    const v3 c = cross(f.ro0, rd0);
    return f.k * dot(c, c);
}

struct RayState {
    v3 ro, rd;
    float travelled;
    float s;
    uint32_t n_rk;
    uint32_t outside;  // 0 / 1: the WGSL's `outside` (:270); u32, so the blackout test stays compare + select
};

// ---- one RK iteration, branch-free ---------------------------------------------------------------
//
// Ops supplies sqrt / length / sdf / rd_derivative / x/6 for the math mode:
//   exact: XOps<true>  correctly rounded cores + domain guard (bh_crmath.hpp);
//          XOps<false> plain IEEE ops (the guard's fallback);  both = the oracle's arithmetic;
//   fast:  FOps        hardware rsq / sqrt, FMA contraction.
// The early exits of the loop body (:272-288) are predicates and the state update is a select, so a
// whole iteration is one basic block: the pair schedule interleaves two rays' iterations and the
// scheduler fills each ray's dependency stalls with the other's instructions.

#if BH_FAST
struct FOps {
    bool bad = false;  // no guard in fast mode
    __device__ __forceinline__ float sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }  // raw v_sqrt_f32
    __device__ __forceinline__ float length(v3 p) { return __builtin_amdgcn_sqrtf(dot(p, p)); }
    template <int K>
    __device__ __forceinline__ v3 div6(v3 x) { return muls(x, 1.0f / 6.0f); }
    __device__ __forceinline__ v3 add2(v3 a, v3 b) {  // a + 2b
        return mk(__builtin_fmaf(2.0f, b.x, a.x), __builtin_fmaf(2.0f, b.y, a.y), __builtin_fmaf(2.0f, b.z, a.z));
    }
    __device__ __forceinline__ v3 ro_half(v3 ro, v3 k) {  // ro + 0.5 k
        return mk(__builtin_fmaf(0.5f, k.x, ro.x), __builtin_fmaf(0.5f, k.y, ro.y), __builtin_fmaf(0.5f, k.z, ro.z));
    }
    __device__ __forceinline__ v3 rd_half(v3 rd, v3 k) { return ro_half(rd, k); }
    __device__ __forceinline__ float sqrt_y(float x, float&) { return __builtin_amdgcn_sqrtf(x); }
    template <int K>
    __device__ __forceinline__ v3 accel_qs(v3 p, float s, float q, float, float = 0.0f) {
        const float iq = rsq(q), iq2 = iq * iq;
        return muls(p, s * (iq2 * iq2 * iq));
    }
    template <int K>
    __device__ __forceinline__ v3 accel(v3 p, float s) { return accel_qs<K>(p, s, dot(p, p), 0.0f); }
    __device__ __forceinline__ void sq_args(float, float) {}
    __device__ __forceinline__ void sq_arg(float) {}
    __device__ __forceinline__ void sdf_args(v3, float&, float&, float&) {}
    __device__ __forceinline__ float sdf_from(v3 p, float rs, uint32_t flags, float, float, float) {
        const float rho = __builtin_amdgcn_sqrtf(p.x * p.x + p.z * p.z);
        const float disc = fmaxf(fmaxf(rho - 6.0f * rs, -(rho - 3.0f * rs)), fabsf(p.y) - 0.02f);
        // min of the four sphere SDFs == sqrt(min of squared distances) - 0.5 (sqrt is monotone)
        const float ay = fabsf(p.y) - 10.0f, ax = fabsf(p.x) - 10.0f, dz = p.z + 10.0f;
        const float m = __builtin_amdgcn_sqrtf(fminf(p.x * p.x + ay * ay, ax * ax + p.y * p.y) + dz * dz) - 0.5f;
        return fminf((flags & BH_SCENE_DISC) ? disc : __builtin_inff(),
                     (flags & BH_SCENE_MARKERS) ? m : __builtin_inff());
    }
};
#else
// Exact mode.  The arithmetic is the normative op sequence of oracle/bh_oracle.c: every rounding
// the same as IEEE f32 evaluated in WGSL source order.  CR = true evaluates the divisions and
// square roots with the cheap correctly rounded cores of bh_crmath.hpp and raises `bad` for any
// operand outside their proven domain; CR = false is plain IEEE ops (hipcc's expansions).  Both
// produce identical bits wherever `bad` stays false.
template <bool CR>
struct XOps {
    static constexpr bool kCR = CR;
    bool bad = false;
    // Numerator domain of the division cores: 0 or >= DIV_N_MIN in magnitude, held to the stricter
    // ACC_N_MIN for the acceleration numerators (rd_half's premise).  Zeros are legal (the
    // cores are exact for them) and occur in two places:
    //  * k1's numerators s*ro: camera-A rays start on two coordinate planes.  Checked through
    //    crm::key (zeros map high, tiny values low): one v_lshl_add per value + v_min3_u32;
    //  * the x/6 numerators when dt == 0 exactly (a ray frozen on the photon-sphere marker): all RK
    //    sums are then +-0.
    // Everywhere else a zero numerator needs an exact cancellation, so those are checked as a float
    // min |n| (one v_min3_f32 with |.| modifiers per three values) and a zero just takes the IEEE
    // path; the x/6 check is waived when dt == 0.  (min |n| everywhere: measured 7 % slower, frozen
    // rays fell back at every step.)
    // Each accumulator is one running chain started by its first value (an explicit +inf start is
    // not folded away, since fminf(inf, NaN) is not NaN), so consecutive values pair up into
    // v_min3_f32: -5 VALU per step, 0.6 % (A/B r01).  (Pooling the denominators' range checks into
    // one min/max over the squared lengths r^2, |ro - cps|^2 and the k-point dot products -- a range
    // of q that implies Q's -- is 5 VALU fewer again but measured 12 % slower at cap 64 and 512 with
    // the same IEEE re-run count: the compiler then interleaves k3's and k4's rsq/rcp chains; the
    // max-ilp and iterative-ilp scheduling strategies did not recover it.  Round 3, with machine
    // scheduling off: one unsigned v_min3_u32 / v_max3_u32 pool over the bit patterns of r^2, rho^2,
    // the marker and photon-sphere arguments and the k-point q's, range [2^-16, 2^24] (implies every
    // root's and Q's domain), 286 -> 280 VALU per step and the same re-run count
    // (tools/diag_slow.py), measured 3.5 % slower on the headline and 11 % on cap 1000 at one frame
    // per launch (packed tail); a float pool the same; profiles/r03/ab_pool/.)
    uint32_t kmin;  // k1 numerators (keys)
    float amin;     // k2..k4 numerators
    float amin6;    // x/6 numerators
    __device__ __forceinline__ static float absmin3(float m, float x, float y, float z) {
        return fminf(fminf(fminf(m, fabsf(x)), fabsf(y)), fabsf(z));
    }
    __device__ __forceinline__ static float absmin3(float x, float y, float z) {
        return fminf(fminf(fabsf(x), fabsf(y)), fabsf(z));
    }
    // Square roots.  The core is exact for x in [SQRT_MIN, FLT_MAX]; outside that the caller must
    // raise `bad`.  Which check covers which root (one v_cmp per bound, so they are pooled):
    //  * r = |ro| and the pow25 roots of rd_derivative: x < 2^-96 makes q*q underflow to 0 and
    //    x = inf makes it inf, so the denominator Q = (q*q)*sqrt(q) is 0, inf or NaN and
    //    div_d_bad(Q) raises `bad` already.  The step's exit tests (before k1) compare r^2, not r
    //    (step_bf), so a lane that leaves early never reads r;
    //  * rho (disc) and the marker distance: one shared range check on the min and max of their
    //    arguments (sq_args; a flag-disabled term can only cause a spare re-run); the photon-sphere
    //    distance (sq_arg, evaluated after the step's early exits).
    __device__ __forceinline__ float sqrt(float x) {
        if constexpr (CR) return crm::sqrt_core(x);
        else return __builtin_sqrtf(x);
    }
    // sqrt(x), and (CR) the v_rsq estimate the core refined: rd_derivative's reciprocal is seeded from it
    __device__ __forceinline__ float sqrt_y(float x, float& y) {
        if constexpr (CR) {
            const crm::SqrtY r = crm::sqrt_core_y(x);
            y = r.y;
            return r.s;
        } else {
            return __builtin_sqrtf(x);
        }
    }
    __device__ __forceinline__ void sq_args(float a, float b) {
        if constexpr (CR) bad |= crm::sqrt_bad2(a, b);
    }
    __device__ __forceinline__ void sq_arg(float a) {
        if constexpr (CR) bad |= crm::sqrt_bad(a);
    }
    template <int K>  // K = 0 for the first call of a step, 1 for the second
    __device__ __forceinline__ v3 div6(v3 x) {
        if constexpr (CR) {
            amin6 = (K == 0) ? absmin3(x.x, x.y, x.z) : absmin3(amin6, x.x, x.y, x.z);
            return mk(crm::div6(x.x), crm::div6(x.y), crm::div6(x.z));
        } else {
            return mk(x.x / 6.0f, x.y / 6.0f, x.z / 6.0f);
        }
    }
    // a + 2b (the RK4 weights): 2b is exact, so the FMA rounds once exactly like the two IEEE adds
    // whenever 2b does not overflow, which the guarded domain rules out (|p| <= 2^12, dt <= 2^13)
    __device__ __forceinline__ v3 add2(v3 a, v3 b) {
        if constexpr (CR) {
            return mk(__builtin_fmaf(2.0f, b.x, a.x), __builtin_fmaf(2.0f, b.y, a.y), __builtin_fmaf(2.0f, b.z, a.z));
        } else {
            return add(a, smul(2.0f, b));
        }
    }
    // ro + 0.5 k, the RK stage positions of k2 and k3 (:140, :143).  CR: fma(0.5, k, ro), one op per
    // component instead of two, and the same bits on every step whose guard stays clear:
    //  * where 0.5 k is exact (|k| >= 2^-125) both forms round ro + 0.5 k once;
    //  * else |0.5 k| < 2^-126: when |ro_i| >= 2^-100 it is below half an ulp of ro_i and both give ro_i;
    //    when ro_i is 0 or smaller, the stage position is 0 or below 2^-99, so this stage's numerator
    //    s * p_i (|s| <= 2^30 on a clear step) is 0 or below ACC_N_MIN and `amin` raises the guard: the
    //    step re-runs in IEEE ops.
    __device__ __forceinline__ v3 ro_half(v3 ro, v3 k) {
        if constexpr (CR) {
            return mk(__builtin_fmaf(0.5f, k.x, ro.x), __builtin_fmaf(0.5f, k.y, ro.y), __builtin_fmaf(0.5f, k.z, ro.z));
        } else {
            return add(ro, smul(0.5f, k));
        }
    }
    // rd + 0.5 k, the RK stage directions of ro_k2 and ro_k3 (:139, :142), k = rd_k1 or rd_k2 = dt * a.
    // CR: fma(0.5, k, rd), exact on every clear step: the acceleration numerators are 0 or >= 2^-40
    // (ACC_N_MIN, and non-zero for k2) and Q <= 2^60, so a_i is 0 or >= 2^-100, and the guard holds dt
    // to 0 or |dt| >= 2^-25 (step_bf), so k_i is 0 or >= 2^-125: 0.5 k is exact and both forms round the
    // same sum once.
    __device__ __forceinline__ v3 rd_half(v3 rd, v3 k) {
        if constexpr (CR) {
            return mk(__builtin_fmaf(0.5f, k.x, rd.x), __builtin_fmaf(0.5f, k.y, rd.y), __builtin_fmaf(0.5f, k.z, rd.z));
        } else {
            return add(rd, smul(0.5f, k));
        }
    }
    // rd_derivative (:125-127): (s * p) / pow(dot(p,p), 2.5), pow(q, 2.5) := (q*q)*sqrt(q);
    // q and sqrt(q) passed in when already known (k1: q = r^2, sqrt(q) = r).
    // K = 1..4: the RK stage (k1's numerators may be zeros, see above)
    // y: v_rsq(q) from the root of q (sqrt_y); unused (a v_rcp of Q seeds RN(1/Q), see the top of the file)
    template <int K>
    __device__ __forceinline__ v3 accel_qs(v3 p, float s, float q, float sq, float y) {
        const float Q = (q * q) * sq;
        const float nx = s * p.x, ny = s * p.y, nz = s * p.z;
        if constexpr (CR) {
            bad |= crm::div_d_bad(Q);
            if constexpr (K == 1) kmin = crm::kmin3(crm::key(nx), crm::key(ny), crm::key(nz));
            else if constexpr (K == 2) amin = absmin3(nx, ny, nz);
            else amin = absmin3(amin, nx, ny, nz);
            const crm::Rcp R = crm::rcp_refined(Q);
            return mk(crm::div_core(nx, R), crm::div_core(ny, R), crm::div_core(nz, R));
        } else {
            return mk(nx / Q, ny / Q, nz / Q);
        }
    }
    template <int K>
    __device__ __forceinline__ v3 accel(v3 p, float s) {
        const float q = dot(p, p);
        float y = 0.0f;
        const float sq = sqrt_y(q, y);
        return accel_qs<K>(p, s, q, sq, y);
    }
    __device__ __forceinline__ float length(v3 p) { return sqrt(dot(p, p)); }
    // sdf (:119-123); markers: min(sqrt(qi) - 0.5) == sqrt(min qi) - 0.5 exactly (monotone ops)
    // sdf_args: the arguments of its two roots (rho^2, the markers' qm) and y*y; sdf_from: the rest
    __device__ __forceinline__ void sdf_args(v3 p, float& rho2, float& yy, float& qm) {
        rho2 = p.x * p.x + p.z * p.z;
        // The four sphere arguments are q1,2 = (xx + (+-10 - y)^2) + zz and q3,4 = ((+-10 - x)^2 + yy)
        // + zz.  Of each pair only the sphere on the point's side can be the minimum, and its
        // argument is computed from t = RN(10 - |y|) (resp. |x|): RN(-10 - y) = -RN(10 + y) and
        // |10 - y| <= 10 + y for y >= 0 (mirrored for y < 0), and every later op (square, sums) is
        // monotone in |t|, so the rounded q of the near sphere is <= the far one's and equals
        // (xx + t*t) + zz bit for bit.  min(q1..q4) == min(qy, qx): 11 ops instead of 20
        // (tests/test_oracle.py::test_marker_pair_reduction checks the identity).
        const float xx = p.x * p.x;
        yy = p.y * p.y;
        const float dz = -10.0f - p.z, zz = dz * dz;
        const float ty = 10.0f - fabsf(p.y), tx = 10.0f - fabsf(p.x);
        const float qy = (xx + ty * ty) + zz, qx = (tx * tx + yy) + zz;
        qm = fminf(qy, qx);
    }
    // the disc and marker terms of sdf_from one by one (the per-term root-free step)
    __device__ __forceinline__ float disc_from(v3 p, float rs, float rho2) {
        const float rho = sqrt(rho2);
        return fmaxf(fmaxf(rho - 6.0f * rs, -(rho - 3.0f * rs)), fabsf(p.y - 0.0f) - 0.02f);
    }
    __device__ __forceinline__ float mark_from(float qm) { return sqrt(qm) - 0.5f; }
    __device__ __forceinline__ float sdf_from(v3 p, float rs, uint32_t flags, float rho2, float, float qm) {
        const float rho = sqrt(rho2);
        const float disc = fmaxf(fmaxf(rho - 6.0f * rs, -(rho - 3.0f * rs)), fabsf(p.y - 0.0f) - 0.02f);
        const float m = sqrt(qm) - 0.5f;
        // fminf(disc, inf) == disc and fminf(inf, m) == m bit for bit: same result as selecting
        return fminf((flags & BH_SCENE_DISC) ? disc : __builtin_inff(),
                     (flags & BH_SCENE_MARKERS) ? m : __builtin_inff());
    }
};
#endif

// One iteration of the loop body (:266-328) from `in` into `out`.  Returns BH_FATE_* if the ray
// terminates in this iteration (n_rk counts completed RK updates), or 0xFF if it continues.
//
// BRANCHY = true (single-ray schedules): a lane whose ray terminates before the RK update (surface /
// blackout, fate >= BH_FATE_SURFACE) returns at once WITHOUT writing `out`: its final state is `in`
// (only n_rk is read for those fates).  Every other lane gets the whole updated state in `out`.
// `in` is never written, so the caller ping-pongs two states and no register copies are needed
// (the IEEE re-run of march_step_io reads `in` again); the RK block is skipped when every active
// lane terminates.  BRANCHY = false keeps one basic block for the pair schedule: `out` is always
// written (selects).  `in` and `out` may alias only when BRANCHY = false.
// Scene flags: a kernel instantiated for one flag set (SF) drops the per-step flag selects.
constexpr uint32_t SF_DYN = 0xFFFFFFFFu;
// SF_CAM_OUT (with a fixed flag set only): the frame's camera lies outside the unit sphere, so the
// blackout test reduces to `!(r > 1)` (march_slot picks the instantiation per wave).  Every ray starts
// at the camera (:363), so at iteration 0 r > 1, no exit fires and `has_been_outside_eh` becomes true;
// from then on a ray with !(r > 1) returns black through :280-281 whether or not :273-274's
// `dot(rd, ro) < 0` holds.  The step then needs neither that product nor the `outside` state (kept
// at 1): -8 VALU per step.  march_slot also requires |s| <= 2^30 on every lane of the wave (the
// division cores' numerator bound, a per-ray constant), so this step does not re-check it.
constexpr uint32_t SF_CAM_OUT = 0x100u;
constexpr uint32_t sf_scene(uint32_t sf) { return sf == SF_DYN ? SF_DYN : (sf & BH_SCENE_DEFAULT); }
constexpr bool sf_cam_out(uint32_t sf) { return sf != SF_DYN && (sf & SF_CAM_OUT) != 0u; }

// r > 1 for r = RN(sqrt(r2)) exactly when r2 > 1 + 2^-23 (step_bf)
constexpr float R2_GT1 = 0x1.000002p0f;

__device__ __forceinline__ bool fate_before_rk(uint32_t fate) { return fate >= BH_FATE_SURFACE; }

// (Measured and not kept, DESIGN.md §5: a "sticky" root-free test that skips the test after a step that took
// the roots; per-term ballots deciding the all-terms test too, 0.5189 vs 0.5193 ms, profiles/r05/sdf_terms3/;
// terms cleared by the lane's radius alone, 0.5217 -> 0.5261 ms, profiles/r05/sdf_radii/, §5 item 29.)
#ifdef BH_DIAG_SLOW
__device__ uint32_t g_diag_skip_wave_steps, g_diag_all_wave_steps, g_diag_far_wave_steps;
// one count per wave: the lowest active lane adds (a global atomic: a vector memory op)
#define BH_DIAG_SKIP_COUNT()                                                                              \
    do {                                                                                                  \
        if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(__builtin_amdgcn_ballot_w64(true)))          \
            atomicAdd(&g_diag_skip_wave_steps, 1u);                                                       \
    } while (0)
#define BH_DIAG_FAR_COUNT()                                                                               \
    do {                                                                                                  \
        if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(__builtin_amdgcn_ballot_w64(true)))          \
            atomicAdd(&g_diag_far_wave_steps, 1u);                                                        \
    } while (0)
#else
#define BH_DIAG_SKIP_COUNT() do {} while (0)
#define BH_DIAG_FAR_COUNT() do {} while (0)
#endif

#if !BH_FAST
// Does this lane's step have dt == dtm*r (:307-310) and no surface hit (:286-288), whatever its three SDF
// roots are?  From the step's own rounded values (r = RN(sqrt r2), dtr = RN(dtm r), rho2, y*y, the markers'
// qm and the photon sphere's qps, all formed exactly as the full step forms them), with no root:
//   T = RN(1.125 dtr + 0.002);  a distance term d = RN(RN(sqrt v) - c) passes when v >= u*u, u = RN(T + c)
//   (tested as fma(-u, u, v) >= 0: one rounding, which keeps the sign of the exact difference):
//   disc (:121)     rho2 >= (T + RN(6 rs))^2  or  y*y >= (T + 0.02)^2   [disc >= RN(rho - 6rs) and
//                   >= RN(|y| - 0.02): fmaxf is >= each non-NaN operand]
//   markers         qm  >= (T + 0.5)^2        photon sphere (:294)  qps >= (T + 0.075)^2
// Proof that a passing lane has dt == dtr and no surface (exact mode: RN sqrt, IEEE ops; dtm > 0 and
// 0 < rs <= 8, the host's skip_sdf gate, so dtr >= 0 and T >= 0.002 (1 - 2^-24)): u = RN(T + c) >=
// (T + c)(1 - 2^-24), so sqrt v >= (T + c)(1 - 2^-24) (for y*y = RN(y^2) one more factor) and
// RN(sqrt v) >= (T + c)(1 - 2^-22); d >= RN(T - (T + c) 2^-22) >= T (1 - 2^-17.6)
// (c <= 48.0001, T >= 0.00199).  So dist = min of the enabled terms >= that bound >= 0.00199 > MIN_DIST
// (no surface), and 0.9f d >= (0.9f * 1.125) dtr (1 - 2^-17.5) = 1.0125 dtr (1 - 2^-17.5) > dtr, so
// RN(0.9f dist) >= dtr (dtr is a float) and fminf(RN(dist * 0.9), dtr) == dtr.  The terms combine with
// the step's own fmaxf / fminf, so a NaN term is dropped exactly where the step drops that distance (a NaN
// argument makes the step's term NaN too); a NaN T (r or dtr NaN) makes every term NaN and the slack NaN,
// which fails; T = +inf gives -inf (finite v) or NaN (v = +inf) terms, which fail or are dropped.
// In the exact build's core pass a wrong r (r2 outside the root core's domain) also raises the k1
// division guard, so that step re-runs in IEEE ops, where the proof holds as written.
// tests/test_skip.py checks the implication on adversarial samples of the step's float32 arithmetic.
// The same test term by term: each term's slack >= 0 alone proves that term's distance
// >= T (1 - 2^-17.6) by the argument above, so a term whose slack holds can be left out of dist (taken as
// +inf): if it was the minimum, every other term is at least as large and still gives RN(0.9 dist) >= dtr;
// its surface test could not fire; and fminf drops a NaN term exactly as it drops +inf.
// tests/test_skip.py::test_per_term_skip_keeps_dt_and_surface checks every subset of cleared terms.
struct SdfSlack { float disc, mark, ps; };
__device__ __forceinline__ SdfSlack sdf_term_slacks(const MarchArgs& a, uint32_t flags, float dtr, float rho2, float yy,
                                                   float qm, float qps) {
    const float T = __builtin_fmaf(dtr, 1.125f, 0.002f);
    const float u6 = T + 6.0f * a.rs, uy = T + 0.02f;
    // v - u^2 rounded once (fma): its sign is the sign of the exact v - u*u
    float disc = fmaxf(__builtin_fmaf(-u6, u6, rho2), __builtin_fmaf(-uy, uy, yy));
    const float um = T + 0.5f;
    float mark = __builtin_fmaf(-um, um, qm);
    const float up = T + 0.075f;
    float ps = __builtin_fmaf(-up, up, qps);
    if (!(flags & BH_SCENE_DISC)) disc = __builtin_inff();
    if (!(flags & BH_SCENE_MARKERS)) mark = __builtin_inff();
    return {disc, mark, ps};
}
__device__ __forceinline__ float sdf_skip_slack(const SdfSlack& t) { return fminf(fminf(t.disc, t.mark), t.ps); }
#endif

// UNI: every active lane of the wave is at loop iteration `it` (n_rk == it: the ping-pong loop), so the
// cap test is a wave-uniform (scalar) compare.
// TINY (the tail's steps): rd + 0.5 k unfused -- the WGSL's own op order, exact for any dt -- where the fused
// form's premise (|dt| >= 2^-25) would send a step with a tiny dt to the IEEE re-run.  The photon-sphere rays whose steps shrink below 2^-25 without
// settling into an exact cycle take hundreds of such steps (camera B: 42 rays, ~210 tiny steps each).
template <bool BRANCHY, class Ops, uint32_t SF = SF_DYN, bool UNI = false, bool TINY = false>
__device__ __forceinline__ bool step_bf(const MarchArgs& a, const Frame& f, const RayState& in, RayState& out, Ops& X,
                                        uint32_t& fate, uint32_t it = 0u) {
    constexpr uint32_t SFS = sf_scene(SF);
    constexpr bool CO = sf_cam_out(SF);
    const uint32_t scene_flags = (SFS == SF_DYN) ? a.scene_flags : SFS;
    const v3 ro = in.ro, rd = in.rd;
    const float travelled = in.travelled, s = in.s;
    const uint32_t n_rk = in.n_rk;
    const float r2 = dot(ro, ro);
    float y1 = 0.0f;                                                   // v_rsq(r2): k1's reciprocal seed
    const float r = X.sqrt_y(r2, y1);                                  // :271
    // :272-283: blackout if (r < 1 and rd.ro < 0), or if !(r > 1) and the ray was outside before;
    // r > 1 sets `outside`.  Bitwise (not short-circuit) logic: lane masks, no branches.
    // The tests read r^2: for r = RN(sqrt(r2)),  r < 1  <=>  r2 < 1  and  r > 1  <=>  r2 > 1 + 2^-23
    // (RN(sqrt) is monotone; sqrt(1 + 2^-23) < 1 + 2^-24, the midpoint above 1, and
    // sqrt(next float) > it; NaN fails every compare either way; tests/test_oracle.py checks every
    // float in [1/4, 4]).  So the exits do not wait for the root, and lanes that leave here need no
    // guard on it.
    const bool bo_on = a.blackout_eh != 0u;
    const bool not_out = !(r2 > R2_GT1);                               // NaN: "else" branch, as the WGSL
    // rd.ro < 0 only matters for lanes inside r < 1 (the black hole's interior: rare).  Written
    // behind a wave-uniform test; the compiler still speculates the product into the step and
    // selects on the test (s_cselect), but the resulting schedule measured 0.7 % faster than the
    // unconditional form (A/B r01, two pairs).  Forcing a real branch materialises the predicates as
    // integers in VGPRs (+8 VALU): slower.
    bool blackout;
    if constexpr (CO) {
        blackout = bo_on & not_out;  // `outside` is 1 from iteration 0 on (SF_CAM_OUT)
    } else {
        bool ingoing = false;
        if (__builtin_amdgcn_ballot_w64(bo_on & (r2 < 1.0f)) != 0ull) ingoing = dot(rd, ro) < 0.0f;
        blackout = bo_on & (((r2 < 1.0f) & ingoing) | (not_out & (in.outside != 0u)));
    }
    float rho2, yy, qm;
    const float dtr = a.dtm * r;                                       // :307-310's second operand
    float dt;
    bool surface = false;
#if !BH_FAST
    // Far field: a lane with a.far_r2 <= r^2 <= FLT_MAX (the host's sdf_far_r2, +inf when off) is so far
    // from the disc, the markers and the photon sphere that every distance term exceeds the root-free
    // test's threshold by construction (proof at sdf_far_r2, bh_host.cpp): when every lane that stays is
    // there, the wave forms no SDF argument at all.  (r^2 = +inf is excluded: there dtm r is +inf while a
    // distance term may stay finite.)
    if (BRANCHY && __builtin_amdgcn_ballot_w64(!(r2 >= a.far_r2 && r2 <= 0x1.fffffep127f) & !blackout) == 0ull) {
        BH_DIAG_FAR_COUNT();
        if (blackout) {
            fate = (uint32_t)BH_FATE_BLACKOUT;
            return true;
        }
        dt = dtr;
    } else
#endif
    {
    X.sdf_args(ro, rho2, yy, qm);                                      // the SDF roots' arguments
#if !BH_FAST
    // Root-free step (BRANCHY): dt = min(0.9 dist, dtm r) needs dist only where it could fall below
    // dtm r / 0.9, and the surface test only below MIN_DIST.  sdf_skip decides "dt == dtm r, no surface"
    // from the squared arguments; when it holds on every live lane (blackout lanes leave either way)
    // the wave skips the three roots, their guards and the distance arithmetic.  Same bits: see sdf_skip.
    // The photon-sphere argument (:294) is formed before the exits for the test.
    if constexpr (BRANCHY) {
        const v3 dc = sub(f.cps, ro);
        const float qps = dot(dc, dc);
        // lanes that need the roots: slack < 0 or NaN, except those that leave by the blackout exit.  (The
        // blackout select becomes a branch around the test.  Taking the lane mask straight from the compare,
        // llvm.amdgcn.fcmp, and masking the blackout lanes as integers is 4 VALU fewer and measured 0.9 %
        // slower: profiles/r04/ab_skip_forms/.)
        const SdfSlack terms = sdf_term_slacks(a, scene_flags, dtr, rho2, yy, qm, qps);
        const float slack = blackout ? __builtin_inff() : sdf_skip_slack(terms);
        const bool fast = a.skip_sdf != 0u && __builtin_amdgcn_ballot_w64(!(slack >= 0.0f)) == 0ull;
        if (fast) {
            BH_DIAG_SKIP_COUNT();
            if (blackout) {
                fate = (uint32_t)BH_FATE_BLACKOUT;
                return true;
            }
            dt = dtr;
        } else if (a.skip_sdf != 0u) {
            // per term: a root only where some lane that stays needs it (sdf_term_slacks); where the disc
            // and markers both clear, the photon sphere alone keeps the wave here (about 98 % of these
            // wave-steps clear it, and 80 % one of the other two: tools/skip_sim.py)
            const bool stay = !blackout;
            const bool nd = __builtin_amdgcn_ballot_w64(stay & !(terms.disc >= 0.0f)) != 0ull;
            const bool nm = __builtin_amdgcn_ballot_w64(stay & !(terms.mark >= 0.0f)) != 0ull;
            const bool np = __builtin_amdgcn_ballot_w64(stay & !(terms.ps >= 0.0f)) != 0ull;
            float dv = __builtin_inff(), mv = __builtin_inff();
            if (nd) {
                dv = X.disc_from(ro, a.rs, rho2);
                X.sq_arg(rho2);
            }
            if (nm) {
                mv = X.mark_from(qm);
                X.sq_arg(qm);
            }
            const float ds = fminf((scene_flags & BH_SCENE_DISC) ? dv : __builtin_inff(),
                                   (scene_flags & BH_SCENE_MARKERS) ? mv : __builtin_inff());  // :285
            if (blackout | (ds < MIN_DIST)) {                            // :286-288
                fate = blackout ? (uint32_t)BH_FATE_BLACKOUT : (uint32_t)BH_FATE_SURFACE;
                return true;
            }
            float dps = __builtin_inff();
            if (np) {
                dps = X.sqrt(qps) - 0.075f;
                X.sq_arg(qps);
            }
            const float dist = fminf(ds, dps);                           // :299
            dt = fminf(dist * 0.9f, dtr);                                // :307-310
        } else {
            const float ds = X.sdf_from(ro, a.rs, scene_flags, rho2, yy, qm);  // :285
            if constexpr (SFS == SF_DYN || SFS == BH_SCENE_DEFAULT) X.sq_args(rho2, qm);
            else if constexpr (SFS == BH_SCENE_DISC) X.sq_arg(rho2);
            else if constexpr (SFS == BH_SCENE_MARKERS) X.sq_arg(qm);
            if (blackout | (ds < MIN_DIST)) {                            // :286-288
                fate = blackout ? (uint32_t)BH_FATE_BLACKOUT : (uint32_t)BH_FATE_SURFACE;
                return true;
            }
            const float dps = X.sqrt(qps) - 0.075f;
            X.sq_arg(qps);
            const float dist = fminf(ds, dps);                           // :299
            dt = fminf(dist * 0.9f, dtr);                                // :307-310
        }
    } else
#endif
    {
        const float ds = X.sdf_from(ro, a.rs, scene_flags, rho2, yy, qm);  // :285
        // the root guards of the enabled terms (a disabled term's value is discarded; a kernel built for
        // one flag set drops its arithmetic entirely)
        if constexpr (SFS == SF_DYN || SFS == BH_SCENE_DEFAULT) X.sq_args(rho2, qm);
        else if constexpr (SFS == BH_SCENE_DISC) X.sq_arg(rho2);
        else if constexpr (SFS == BH_SCENE_MARKERS) X.sq_arg(qm);
        surface = ds < MIN_DIST;                                           // :286-288
        if constexpr (BRANCHY) {
            if (blackout | surface) {
                fate = blackout ? (uint32_t)BH_FATE_BLACKOUT : (uint32_t)BH_FATE_SURFACE;
                return true;
            }
        }
        // :294 after the exits (measured: 1.5 % faster than before them, A/B r01; neutral without
        // machine scheduling)
        const v3 dc = sub(f.cps, ro);
        const float qps = dot(dc, dc);
        const float dps = X.sqrt(qps) - 0.075f;
        X.sq_arg(qps);
        const float dist = fminf(ds, dps);                                 // :299
        dt = fminf(dist * 0.9f, dtr);                                      // :307-310
    }
    }
    // get_delta_photon_rk4 (:134-151).  UNF (the tail's steps, TINY): rd + 0.5 k as its two IEEE ops, the WGSL's
    // order, exact for any dt (XOps::rd_half's fma equals it only for |dt| >= 2^-25); the rest keeps the cores
    // and their guards (the x/6 core's domain, |x| >= 2^-60, is checked as always).
    v3 dro, drd;
    auto rk_update = [&](auto UNFc) {
        constexpr bool UNF = decltype(UNFc)::value;
        auto rd_half = [&](v3 v, v3 k) { return UNF ? add(v, smul(0.5f, k)) : X.rd_half(v, k); };
        const v3 ro_k1 = smul(dt, rd);
        const v3 rd_k1 = smul(dt, X.template accel_qs<1>(ro, s, r2, r, y1));
        const v3 ro_k2 = smul(dt, rd_half(rd, rd_k1));
        const v3 rd_k2 = smul(dt, X.template accel<2>(X.ro_half(ro, ro_k1), s));
        const v3 ro_k3 = smul(dt, rd_half(rd, rd_k2));
        const v3 rd_k3 = smul(dt, X.template accel<3>(X.ro_half(ro, ro_k2), s));
        const v3 ro_k4 = smul(dt, add(rd, rd_k3));
        const v3 rd_k4 = smul(dt, X.template accel<4>(add(ro, ro_k3), s));
        const v3 sro = add(X.add2(X.add2(ro_k1, ro_k2), ro_k3), ro_k4);
        const v3 srd = add(X.add2(X.add2(rd_k1, rd_k2), rd_k3), rd_k4);
        dro = X.template div6<0>(sro);
        drd = X.template div6<1>(srd);
#if !BH_FAST
        if constexpr (Ops::kCR) {
            // Domain of the division cores: every numerator is 0 or >= 2^-60 in magnitude, and
            // |s| <= 2^30, which with Q <= 2^60 (|p| <= 2^12) bounds every |s*p_i| <= 2^42.
            X.bad |= X.kmin < crm::KEY_ACC_MIN;
            X.bad |= !(X.amin >= crm::ACC_N_MIN);
            if constexpr (!UNF) X.bad |= (fabsf(dt) < 0x1p-25f) & (dt != 0.0f);  // rd_half's premise
            X.bad |= !(X.amin6 >= crm::DIV_N_MIN) & (dt != 0.0f);
            if constexpr (!CO) X.bad |= !(fabsf(s) <= 0x1p30f);  // SF_CAM_OUT: checked once per wave
        }
#endif
    };
#if BH_FAST
    rk_update(std::false_type{});
#else
    rk_update(std::bool_constant<TINY && Ops::kCR>{});
#endif
    const v3 nro = add(ro, dro), nrd = add(rd, drd);                   // :315, :322
    const float ntr = travelled + dt;                                  // :324
    out.s = s;
    out.outside = CO ? 1u : (not_out ? in.outside : 1u);               // only read when bo_on
    const bool escape = ntr > a.max_dist;                              // :325-327
    const bool capped = (UNI ? it : n_rk) + 1u >= a.max_iters;         // loop end (:266)
    if constexpr (BRANCHY) {
        out.ro = nro;
        out.rd = nrd;
        out.travelled = ntr;
        out.n_rk = n_rk + 1u;
        fate = escape ? (uint32_t)BH_FATE_ESCAPE : (uint32_t)BH_FATE_CAP;
        return escape | capped;
    }
    const bool pre = blackout | surface;
    const bool go = !pre;
    out.ro = sel(go, nro, ro);
    out.rd = sel(go, nrd, rd);
    out.travelled = go ? ntr : travelled;
    out.n_rk = n_rk + (go ? 1u : 0u);
    // flat selects (a nested ?: becomes exec-mask branches)
    const uint32_t pre_fate = blackout ? (uint32_t)BH_FATE_BLACKOUT : (uint32_t)BH_FATE_SURFACE;
    const uint32_t post_fate = escape ? (uint32_t)BH_FATE_ESCAPE : (uint32_t)BH_FATE_CAP;
    fate = go ? post_fate : pre_fate;
    return pre | escape | capped;
}

#ifdef BH_DIAG_SLOW
__device__ uint32_t g_diag_slow_lane_steps, g_diag_slow_wave_steps;  // (g_diag_skip/all_wave_steps above)
#endif

#ifndef BH_TAIL_PACKED
#define BH_TAIL_PACKED 0
#endif
#if !BH_FAST && BH_TAIL_PACKED
// ---- the tail's step, in packed FP32 (exact mode) ---------------------------------------------------
// The same arithmetic as step_bf<true, XOps<true>> -- every rounding identical, in the same order, the
// same guards -- with the x and y components of each vector in one 64-bit register pair, so that one
// v_pk_{add,mul,fma}_f32 does both.  It runs only in the cycle-watch loop (march_cycles), i.e. in waves
// still marching after PRIO_ITERS iterations, which are few per SIMD: a wave alone issues a packed op
// in the slot of a scalar one (tools/ubench/lone_wave.hip: 4.6 vs 4.7 cycles, profiles/r02/lone_wave.log),
// so the tail's serial step chain gets shorter; at 8 waves per SIMD a packed op costs more than two
// scalar ones (5.7 vs 2 x 2.3 cycles), so the bulk keeps the scalar step.
typedef float f2 __attribute__((ext_vector_type(2)));
struct p3 { f2 xy; float z; };
__device__ __forceinline__ p3 pk(v3 a) { return {f2{a.x, a.y}, a.z}; }
__device__ __forceinline__ v3 unpk(p3 a) { return mk(a.xy.x, a.xy.y, a.z); }
__device__ __forceinline__ f2 bc(float s) { return f2{s, s}; }
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ p3 padd(p3 a, p3 b) { return {a.xy + b.xy, a.z + b.z}; }
__device__ __forceinline__ p3 psub(p3 a, p3 b) { return {a.xy - b.xy, a.z - b.z}; }
__device__ __forceinline__ p3 psmul(float s, p3 a) { return {bc(s) * a.xy, s * a.z}; }  // s*x == x*s
// dot(a, b) = (a.x*b.x + a.y*b.y) + a.z*b.z
__device__ __forceinline__ float pdot(p3 a, p3 b) {
    const f2 m = a.xy * b.xy;
    return (m.x + m.y) + a.z * b.z;
}
// div_core of the three components by one refined reciprocal
__device__ __forceinline__ p3 pdiv(p3 n, const crm::Rcp& R) {
    const p3 y{n.xy * bc(R.r), n.z * R.r};
    const p3 e{pfma(bc(R.d), y.xy, -n.xy), __builtin_fmaf(R.d, y.z, -n.z)};
    return {pfma(-e.xy, bc(R.r), y.xy), __builtin_fmaf(-e.z, R.r, y.z)};
}
__device__ __forceinline__ p3 pdiv6(p3 x) {  // crm::div6 per component
    return {pfma(x.xy, bc(crm::R6_H), x.xy * bc(crm::R6_L)), crm::div6(x.z)};
}
__device__ __forceinline__ p3 pro_half(p3 ro, p3 k) {  // ro + 0.5 k, as XOps<true>::ro_half
    return {pfma(bc(0.5f), k.xy, ro.xy), __builtin_fmaf(0.5f, k.z, ro.z)};
}
__device__ __forceinline__ p3 padd2(p3 a, p3 b) {  // a + 2b, as XOps<true>::add2
    return {pfma(bc(2.0f), b.xy, a.xy), __builtin_fmaf(2.0f, b.z, a.z)};
}

struct PkGuard {
    bool bad = false;
    uint32_t kmin;
    float amin, amin6;
};

// rd_derivative as XOps<true>::accel_qs<K>
template <int K>
__device__ __forceinline__ p3 paccel_qs(p3 p, float s, float q, float sq, float y, PkGuard& G) {
    const float Q = (q * q) * sq;
    const p3 n = psmul(s, p);
    G.bad |= crm::div_d_bad(Q);
    if constexpr (K == 1) G.kmin = crm::kmin3(crm::key(n.xy.x), crm::key(n.xy.y), crm::key(n.z));
    else if constexpr (K == 2) G.amin = XOps<true>::absmin3(n.xy.x, n.xy.y, n.z);
    else G.amin = XOps<true>::absmin3(G.amin, n.xy.x, n.xy.y, n.z);
    return pdiv(n, crm::rcp_refined(Q));
}
template <int K>
__device__ __forceinline__ p3 paccel(p3 p, float s, PkGuard& G) {
    const float q = pdot(p, p);
    const crm::SqrtY sy = crm::sqrt_core_y(q);
    return paccel_qs<K>(p, s, q, sy.s, sy.y, G);
}

// step_bf<true, XOps<true>, SF> with packed pairs (see above): same contract (`out` is not written for
// the fates decided before the RK update), `G.bad` set when an operand left a core's domain.
template <uint32_t SF>
__device__ __forceinline__ bool step_tail(const MarchArgs& a, const Frame& f, const RayState& in, RayState& out,
                                          PkGuard& G, uint32_t& fate) {
    constexpr uint32_t SFS = sf_scene(SF);
    constexpr bool CO = sf_cam_out(SF);
    const uint32_t scene_flags = (SFS == SF_DYN) ? a.scene_flags : SFS;
    const p3 ro = pk(in.ro), rd = pk(in.rd);
    const float travelled = in.travelled, s = in.s;
    const uint32_t n_rk = in.n_rk;
    const f2 sq_xy = ro.xy * ro.xy;                 // x*x, y*y
    const float zz0 = ro.z * ro.z;
    const float r2 = (sq_xy.x + sq_xy.y) + zz0;     // dot(ro, ro)
    const crm::SqrtY sy1 = crm::sqrt_core_y(r2);
    const float r = sy1.s;
    const bool bo_on = a.blackout_eh != 0u;
    const bool not_out = !(r2 > R2_GT1);
    bool blackout;
    if constexpr (CO) {
        blackout = bo_on & not_out;
    } else {
        bool ingoing = false;
        if (__builtin_amdgcn_ballot_w64(bo_on & (r2 < 1.0f)) != 0ull) ingoing = pdot(rd, ro) < 0.0f;
        blackout = bo_on & (((r2 < 1.0f) & ingoing) | (not_out & (in.outside != 0u)));
    }
    // sdf (XOps::sdf): disc from rho^2 = x*x + z*z, markers from the near sphere of each pair
    const float rho2 = sq_xy.x + zz0;
    const float rho = crm::sqrt_core(rho2);
    const float disc = fmaxf(fmaxf(rho - 6.0f * a.rs, -(rho - 3.0f * a.rs)), fabsf(ro.xy.y - 0.0f) - 0.02f);
    const float dz = -10.0f - ro.z, zz = dz * dz;
    const f2 t{10.0f - fabsf(ro.xy.x), 10.0f - fabsf(ro.xy.y)};  // (tx, ty)
    const f2 t2 = t * t;                                            // (tx*tx, ty*ty)
    // (qy, qx) = ((xx + ty*ty) + zz, (yy + tx*tx) + zz); tx*tx + yy == yy + tx*tx exactly
    const f2 qyx = (sq_xy + t2.yx) + bc(zz);
    const float qm = fminf(qyx.x, qyx.y);
    const float m = crm::sqrt_core(qm) - 0.5f;
    const float ds = fminf((scene_flags & BH_SCENE_DISC) ? disc : __builtin_inff(),
                           (scene_flags & BH_SCENE_MARKERS) ? m : __builtin_inff());
    if constexpr (SFS == SF_DYN || SFS == BH_SCENE_DEFAULT) G.bad |= crm::sqrt_bad2(rho2, qm);
    else if constexpr (SFS == BH_SCENE_DISC) G.bad |= crm::sqrt_bad(rho2);
    else if constexpr (SFS == BH_SCENE_MARKERS) G.bad |= crm::sqrt_bad(qm);
    const bool surface = ds < MIN_DIST;
    if (blackout | surface) {
        fate = blackout ? (uint32_t)BH_FATE_BLACKOUT : (uint32_t)BH_FATE_SURFACE;
        return true;
    }
    const p3 dc = psub(pk(f.cps), ro);
    const float qps = pdot(dc, dc);
    const float dps = crm::sqrt_core(qps) - 0.075f;
    G.bad |= crm::sqrt_bad(qps);
    const float dist = fminf(ds, dps);
    const float dt = fminf(dist * 0.9f, a.dtm * r);
    // the RK update in the tail's form (step_bf TINY): rd + 0.5 k unfused, exact for any dt
    auto rd_half = [&](p3 v, p3 k) { return padd(v, psmul(0.5f, k)); };
    const p3 ro_k1 = psmul(dt, rd);
    const p3 rd_k1 = psmul(dt, paccel_qs<1>(ro, s, r2, r, sy1.y, G));
    const p3 ro_k2 = psmul(dt, rd_half(rd, rd_k1));
    const p3 rd_k2 = psmul(dt, paccel<2>(pro_half(ro, ro_k1), s, G));
    const p3 ro_k3 = psmul(dt, rd_half(rd, rd_k2));
    const p3 rd_k3 = psmul(dt, paccel<3>(pro_half(ro, ro_k2), s, G));
    const p3 ro_k4 = psmul(dt, padd(rd, rd_k3));
    const p3 rd_k4 = psmul(dt, paccel<4>(padd(ro, ro_k3), s, G));
    const p3 sro = padd(padd2(padd2(ro_k1, ro_k2), ro_k3), ro_k4);
    const p3 srd = padd(padd2(padd2(rd_k1, rd_k2), rd_k3), rd_k4);
    G.amin6 = XOps<true>::absmin3(XOps<true>::absmin3(sro.xy.x, sro.xy.y, sro.z), srd.xy.x, srd.xy.y, srd.z);
    const p3 dro = pdiv6(sro), drd = pdiv6(srd);
    G.bad |= !(G.amin6 >= crm::DIV_N_MIN) & (dt != 0.0f);
    G.bad |= G.kmin < crm::KEY_ACC_MIN;
    G.bad |= !(G.amin >= crm::ACC_N_MIN);
    if constexpr (!CO) G.bad |= !(fabsf(s) <= 0x1p30f);
    const float ntr = travelled + dt;
    out.s = s;
    out.outside = CO ? 1u : (not_out ? in.outside : 1u);
    out.ro = unpk(padd(ro, dro));
    out.rd = unpk(padd(rd, drd));
    out.travelled = ntr;
    out.n_rk = n_rk + 1u;
    const bool escape = ntr > a.max_dist;
    fate = escape ? (uint32_t)BH_FATE_ESCAPE : (uint32_t)BH_FATE_CAP;
    return escape | (n_rk + 1u >= a.max_iters);
}
#endif

// One iteration for one ray from `in` into `out` (step_bf<true> contract: `out` is not written for
// fates before the RK update), with the exact mode's guarded fast path and its rare IEEE re-run.
template <uint32_t SF = SF_DYN, bool UNI = false, bool TINY = false>
__device__ __forceinline__ bool march_step_io(const MarchArgs& a, const Frame& f, const RayState& in, RayState& out,
                                              uint32_t& fate, uint32_t it = 0u) {
#if BH_FAST
    FOps X;
    return step_bf<true, FOps, SF, UNI>(a, f, in, out, X, fate, it);
#else
    XOps<true> X;
#ifdef BH_DIAG_SLOW
    if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(__builtin_amdgcn_ballot_w64(true)))
        atomicAdd(&g_diag_all_wave_steps, 1u);
#endif
    bool done = step_bf<true, XOps<true>, SF, UNI, TINY>(a, f, in, out, X, fate, it);
#ifdef BH_DIAG_SLOW
    const uint64_t badm = __builtin_amdgcn_ballot_w64(X.bad);
    if (badm != 0ull && (threadIdx.x & 63u) == 0u) {
        atomicAdd(&g_diag_slow_wave_steps, 1u);
        atomicAdd(&g_diag_slow_lane_steps, (uint32_t)__popcll(badm));
    }
#endif
    // rare IEEE re-run: a divergent `if` on the guard's lane mask (s_and_saveexec + execz skip; a
    // ballot here costs a v_cndmask + v_cmp per step to materialise the mask)
    if (__builtin_expect(X.bad, 0)) {
        XOps<false> Y;
        done = step_bf<true, XOps<false>, SF, UNI>(a, f, in, out, Y, fate, it);
    }
    return done;
#endif
}

// One iteration of a tail wave (the tile schedule's cycle watch), in place: BH_FATE_* if the ray
// terminates, else 0xFF.  The latency build of the exact kernels (BH_TAIL_PACKED, bh_march_exact_lat.hip)
// runs the packed step, with the same rare IEEE re-run: a lone tail wave's step 0.89 -> 0.79 us, config
// 5 (one frame, cap 1000) 0.824 -> 0.734 ms.  The issue-order build keeps the scalar step: in
// multi-frame launches the tail waves share their SIMDs with other frames' bulk, where a packed op
// costs more than two scalar ones, and the packed tail measured 0.4 % slower there (A/B r02,
// profiles/r02/ab_tail.log).
template <uint32_t SF = SF_DYN>
__device__ __forceinline__ uint32_t march_step_tail(const MarchArgs& a, const Frame& f, RayState& st) {
#if BH_FAST || !BH_TAIL_PACKED
    RayState t = st;
    uint32_t fate;
    const bool done = march_step_io<SF, false, true>(a, f, st, t, fate);
#else
    RayState t = st;
    uint32_t fate;
    PkGuard G;
    bool done = step_tail<SF>(a, f, st, t, G, fate);
    if (__builtin_expect(G.bad, 0)) {
        XOps<false> Y;
        done = step_bf<true, XOps<false>, SF>(a, f, st, t, Y, fate);
    }
#endif
    st = t;
    return done ? fate : 0xFFu;
}

// One iteration for one ray in place (persistent schedule): BH_FATE_* if the ray terminates, else 0xFF.
template <uint32_t SF = SF_DYN>
__device__ __forceinline__ uint32_t march_step(const MarchArgs& a, const Frame& f, RayState& st) {
    // t = st / st = t rather than a select on the fate: the copies fill the tail waves' dependency
    // stalls (a select form measured 9 % slower at cap 1000, A/B r01)
    RayState t = st;  // lanes that leave before the RK update keep `st` (n_rk is what they need)
    uint32_t fate;
    const bool done = march_step_io<SF>(a, f, st, t, fate);
    st = t;
    return done ? fate : 0xFFu;
}

// One iteration for two independent rays of the same lane (pair schedule).  Dead rays (alive_k
// false) are computed on their frozen state and discarded, so the two iterations stay one block.
__device__ __forceinline__ void march_step2(const MarchArgs& a, const Frame& f, RayState& s0, RayState& s1,
                                            bool& alive0, bool& alive1, uint32_t& fate0, uint32_t& fate1) {
    RayState t0, t1;
#if BH_FAST
    FOps X0, X1;
    uint32_t f0, f1;
    const bool d0 = step_bf<false>(a, f, s0, t0, X0, f0);
    const bool d1 = step_bf<false>(a, f, s1, t1, X1, f1);
#else
    XOps<true> X0, X1;
    uint32_t f0, f1;
    bool d0 = step_bf<false>(a, f, s0, t0, X0, f0);
    bool d1 = step_bf<false>(a, f, s1, t1, X1, f1);
    const bool bad0 = X0.bad & alive0, bad1 = X1.bad & alive1;
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(bad0 | bad1) != 0ull, 0)) {   // rare IEEE re-runs
        if (bad0) { XOps<false> Y; d0 = step_bf<false>(a, f, s0, t0, Y, f0); }
        if (bad1) { XOps<false> Y; d1 = step_bf<false>(a, f, s1, t1, Y, f1); }
    }
#endif
    // selects, not branches
    s0.ro = sel(alive0, t0.ro, s0.ro); s0.rd = sel(alive0, t0.rd, s0.rd);
    s0.travelled = alive0 ? t0.travelled : s0.travelled; s0.n_rk = alive0 ? t0.n_rk : s0.n_rk;
    s0.outside = alive0 ? t0.outside : s0.outside;
    s1.ro = sel(alive1, t1.ro, s1.ro); s1.rd = sel(alive1, t1.rd, s1.rd);
    s1.travelled = alive1 ? t1.travelled : s1.travelled; s1.n_rk = alive1 ? t1.n_rk : s1.n_rk;
    s1.outside = alive1 ? t1.outside : s1.outside;
    const bool e0 = alive0 & d0, e1 = alive1 & d1;
    fate0 = e0 ? f0 : fate0;
    fate1 = e1 ? f1 : fate1;
    alive0 = alive0 & !e0;
    alive1 = alive1 & !e1;
}

// Colour of a finished ray (:329-345 for sky rays; :275/:281 blackout -> 0; :287 surface -> 1).
__device__ __forceinline__ v3 shade(const MarchArgs& a, const float* lut, uint32_t fate, v3 rd) {
    if (fate == BH_FATE_BLACKOUT) return mk(0.0f, 0.0f, 0.0f);
    if (fate == BH_FATE_SURFACE) return mk(1.0f, 1.0f, 1.0f);
#if BH_FAST
    const v3 n = normalize(rd);                             // :330
    const float az = atan2f(n.z, n.x);                      // :332
    const float x = (az + ONE_PI) / TWO_PI;                 // :334
#else
    const v3 n = normalize_x(rd);
    // RN_f32 of the f64 atan2 (:332): the short f64 core, and the library call for the lanes whose angle
    // lies too close to an f32 rounding midpoint for the core to decide (about 2^-21 of them)
    const crm::Atan2 at = crm::atan2_core(n.z, n.x);
    float az = at.f;
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(at.near) != 0ull, 0)) {
        if (at.near) az = (float)atan2((double)n.z, (double)n.x);
    }
    // az + pi is +0 or in [2^-22, 7] (az is an f32 in [-RN(pi), RN(pi)]): inside the division core's
    // domain
    const float x = crm::div_core(az + ONE_PI, crm::Rcp{TWO_PI, 1.0f / TWO_PI});  // RN(1/2pi) folded
#endif
    const float y = (n.y + 1.0f) * 0.5f;                    // :336
    v3 col = sample_sky(a, lut, x, 1.0f - y);               // :341
#if BH_FAST
    col.y = col.y * __builtin_sqrtf(col.y);                 // :342
    col.z = col.z * __builtin_sqrtf(col.z);                 // :343
#else
    col.y = pow15_x(col.y);
    col.z = pow15_x(col.z);
#endif
    return col;
}

#ifndef BH_SKY_LDS
#define BH_SKY_LDS 0
#endif
#if BH_SKY_LDS && !BH_FAST
// A/B variant (north_star's "sky texture tile-staged through LDS"): shade() for a whole
// tile wave, whose rays' bilinear footprints usually fall in a few texels of the sky.  When every sky
// lane's 2x2 footprint lies in the 8x8 texel box around the first sky lane's, the wave stages that box
// into LDS (one texel per lane, the wave's 4 KiB history area, free after the march) and each lane reads
// its four texels from there; otherwise (and in partial tiles) the texels come from global memory as in
// sample_sky.  The decode and lerps are sample_sky's, so the bits are the same.  Full exec required.
__device__ __forceinline__ v3 shade_tile(const MarchArgs& a, const float* lut, uint32_t fate, v3 rd, uint32_t* S,
                                         uint32_t lane) {
    const bool sky = (fate != BH_FATE_BLACKOUT) & (fate != BH_FATE_SURFACE);
    float u = 0.0f, v = 0.0f;
    if (sky) {
        const v3 n = normalize_x(rd);
        const crm::Atan2 at = crm::atan2_core(n.z, n.x);
        float az = at.f;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(at.near) != 0ull, 0)) {
            if (at.near) az = (float)atan2((double)n.z, (double)n.x);
        }
        u = crm::div_core(az + ONE_PI, crm::Rcp{TWO_PI, 1.0f / TWO_PI});
        v = 1.0f - (n.y + 1.0f) * 0.5f;
    }
    const bool nan = (u != u) | (v != v);  // Q8: texel (0, 0)
    float tx = u * (float)a.sky_w - 0.5f;
    float ty = v * (float)a.sky_h - 0.5f;
    tx = fminf(fmaxf(tx, -1.0f), (float)a.sky_w);
    ty = fminf(fmaxf(ty, -1.0f), (float)a.sky_h);
    const float fx0 = floorf(tx), fy0 = floorf(ty);
    const float fa = tx - fx0, fb = ty - fy0;
    const int32_t wm = (int32_t)a.sky_w - 1, hm = (int32_t)a.sky_h - 1;
    int32_t x0 = (int32_t)fx0, y0 = (int32_t)fy0;
    int32_t x1 = clampi(x0 + 1, 0, wm), y1 = clampi(y0 + 1, 0, hm);
    x0 = clampi(x0, 0, wm);
    y0 = clampi(y0, 0, hm);
    if (nan) { x0 = x1 = 0; y0 = y1 = 0; }
    const bool need = sky;
    bool staged = false;
    int32_t bx = 0, by = 0;
    if (__builtin_amdgcn_read_exec() == ~0ull) {  // a full tile wave (wave-uniform)
        const uint64_t nm = __builtin_amdgcn_ballot_w64(need);
        if (nm != 0ull) {
            const int lead = __builtin_ctzll(nm);
            bx = __builtin_amdgcn_readlane(x0, lead) - 3;
            by = __builtin_amdgcn_readlane(y0, lead) - 3;
            const bool in = !need | ((x0 >= bx) & (x1 <= bx + 7) & (y0 >= by) & (y1 <= by + 7));
            if (__builtin_amdgcn_ballot_w64(!in) == 0ull) {
                const int32_t sx = clampi(bx + (int32_t)(lane & 7u), 0, wm), sy = clampi(by + (int32_t)(lane >> 3), 0, hm);
                S[lane] = a.sky[(size_t)sy * a.sky_w + (size_t)sx];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                staged = true;
            }
        }
    }
    if (!sky) return fate == BH_FATE_SURFACE ? mk(1.0f, 1.0f, 1.0f) : mk(0.0f, 0.0f, 0.0f);
    uint32_t w00, w10, w01, w11;
    if (staged) {
        const int32_t o = (y0 - by) * 8 + (x0 - bx), dx = x1 - x0, dy = (y1 - y0) * 8;
        w00 = S[o]; w10 = S[o + dx]; w01 = S[o + dy]; w11 = S[o + dy + dx];
    } else {
        w00 = texel_u32(a, x0, y0); w10 = texel_u32(a, x1, y0); w01 = texel_u32(a, x0, y1); w11 = texel_u32(a, x1, y1);
    }
    v3 col;
    if (nan) {
        col = decode(lut, w00);
    } else {
        const v3 t00 = decode(lut, w00), t10 = decode(lut, w10), t01 = decode(lut, w01), t11 = decode(lut, w11);
        const float ia = 1.0f - fa, ib = 1.0f - fb;
        const v3 top = add(muls(t00, ia), muls(t10, fa));
        const v3 bot = add(muls(t01, ia), muls(t11, fa));
        col = add(muls(top, ib), muls(bot, fb));
    }
    col.y = pow15_x(col.y);
    col.z = pow15_x(col.z);
    return col;
}
#endif

// Output texel store; the format is a template parameter (one kernel instantiation per format keeps
// the BGRA8 encoder out of the other formats' code: it measured 1.8 % on the RGBA16F kernel).
template <uint32_t FMT>
__device__ __forceinline__ void store_px(void* base, size_t idx, v3 c, const float* enc) {
    if constexpr (FMT == BH_OUT_RGBA32F) {
        reinterpret_cast<float4*>(base)[idx] = make_float4(c.x, c.y, c.z, 1.0f);
    } else if constexpr (FMT == BH_OUT_RGBA16F) {
        __half2 lo = __floats2half2_rn(c.x, c.y);
        __half2 hi = __floats2half2_rn(c.z, 1.0f);
        uint2 w;
        w.x = *reinterpret_cast<uint32_t*>(&lo);
        w.y = *reinterpret_cast<uint32_t*>(&hi);
        reinterpret_cast<uint2*>(base)[idx] = w;
    } else {
        static_assert(FMT == BH_OUT_BGRA8_SRGB, "output format");
        reinterpret_cast<uint32_t*>(base)[idx] = srgb_bgra8(c.x, c.y, c.z, enc);
    }
}

// LDS tables of a workgroup: [0, 256) the sRGB decode of sky texels, then for BGRA8 output the
// encoder's 257 thresholds.  NT = the workgroup's threads (a divisor or multiple of 256).
template <uint32_t FMT>
constexpr int lds_tables() { return FMT == BH_OUT_BGRA8_SRGB ? 256 + SRGB_TABLE : 256; }
template <uint32_t FMT, uint32_t NT = 256>
__device__ __forceinline__ void load_tables(const MarchArgs& a, float* tab) {
#pragma unroll
    for (uint32_t i = threadIdx.x; i < 256u; i += NT) {
        tab[i] = a.srgb_lut[i];
        if constexpr (FMT == BH_OUT_BGRA8_SRGB) tab[256 + i] = a.srgb_enc[i];
    }
    if constexpr (FMT == BH_OUT_BGRA8_SRGB)
        if (threadIdx.x == 0) tab[256 + 256] = a.srgb_enc[256];
}

// BH_LAYOUT_TILES_RGB(M) store: pixel idx = tile * 64 + lane goes to three channel planes of its tile
// (alpha, always 1, is dropped; the unpack restores it).  Each plane store of a wave is one
// contiguous 64-element run.  TE = the tile's size in channel elements (192, or 192 + the 8-byte
// blackout mask word of BH_LAYOUT_TILES_RGBM).
template <uint32_t FMT, uint32_t TE>
__device__ __forceinline__ void store_px_planar(void* base, size_t idx, v3 c, const float* enc) {
    const size_t o = (idx >> 6) * TE + (idx & 63u);
    if constexpr (FMT == BH_OUT_RGBA32F) {
        float* p = reinterpret_cast<float*>(base) + o;
        p[0] = c.x; p[64] = c.y; p[128] = c.z;
    } else if constexpr (FMT == BH_OUT_RGBA16F) {
        __half* p = reinterpret_cast<__half*>(base) + o;
        p[0] = __float2half_rn(c.x); p[64] = __float2half_rn(c.y); p[128] = __float2half_rn(c.z);
    } else {
        const uint32_t w = srgb_bgra8(c.x, c.y, c.z, enc);
        uint8_t* p = reinterpret_cast<uint8_t*>(base) + o;
        p[0] = (uint8_t)w; p[64] = (uint8_t)(w >> 8); p[128] = (uint8_t)(w >> 16);
    }
}

// Channel elements of one BH_LAYOUT_TILES_RGBM tile: three planes of 64, then the 8-byte mask word.
template <uint32_t FMT>
constexpr uint32_t rgbm_tile_elems() { return 192u + 8u / (FMT == BH_OUT_RGBA32F ? 4u : FMT == BH_OUT_RGBA16F ? 2u : 1u); }

// BH_LAYOUT_TILES_RGBM14 store (include/bh_render.h): the RGBA16F channels, each an fp16 in [0, 1] (bits
// 14-15 zero), as 64 words r | g << 14 | (b & 0xF) << 28, 64 bytes (b >> 4) & 0xFF, the wave's ballots of
// b's bits 12 and 13, and the blackout mask word -- 86 words per tile.  Every active lane of the wave
// must hold a pixel of the same tile (as for RGBM); its first active lane stores the three 64-bit words.
__device__ __forceinline__ void store_rgbm14(void* base, size_t idx, v3 c, bool zero) {
    const uint32_t r = __half_as_ushort(__float2half_rn(c.x)), g = __half_as_ushort(__float2half_rn(c.y));
    const uint32_t b = __half_as_ushort(__float2half_rn(c.z));
    uint32_t* W = reinterpret_cast<uint32_t*>(base) + (idx >> 6) * 86u;
    const uint32_t e = (uint32_t)idx & 63u;
    W[e] = r | (g << 14) | (b << 28);
    reinterpret_cast<uint8_t*>(W + 64)[e] = (uint8_t)(b >> 4);
    const uint64_t m12 = __builtin_amdgcn_ballot_w64(((b >> 12) & 1u) != 0u);
    const uint64_t m13 = __builtin_amdgcn_ballot_w64(((b >> 13) & 1u) != 0u);
    const uint64_t mz = __builtin_amdgcn_ballot_w64(zero);
    if (e == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec())) {
        uint64_t* M = reinterpret_cast<uint64_t*>(W + 80);
        M[0] = m12;
        M[1] = m13;
        M[2] = mz;
    }
}

// fs_main output (:365-369): col, blackout_col = dot(col,col) < 1 ? 0 : col, debug counters.
// BH_LAYOUT_TILES_RGBM: every active lane of the calling wave must hold a pixel of the same tile
// (true of the tile and pair schedules, bh_render rejects the others): the wave's ballot of the
// blackout test is the tile's mask word, stored by its first active lane.
template <uint32_t FMT>
__device__ __forceinline__ void write_pixel(const MarchArgs& a, const float* tab, size_t idx, v3 col, uint32_t n_rk,
                                            uint32_t fate, uint32_t steps) {
    const bool zero = dot(col, col) < 1.0f;
    const v3 bo = zero ? mk(0.0f, 0.0f, 0.0f) : col;
    if (a.layout == BH_LAYOUT_TILES_RGB) {
        store_px_planar<FMT, 192u>(a.out_col, idx, col, tab + 256);
        if (a.out_blackout) store_px_planar<FMT, 192u>(a.out_blackout, idx, bo, tab + 256);
    } else if (a.layout == BH_LAYOUT_TILES_RGBM) {
        constexpr uint32_t TE = rgbm_tile_elems<FMT>();
        constexpr uint32_t CB = FMT == BH_OUT_RGBA32F ? 4u : FMT == BH_OUT_RGBA16F ? 2u : 1u;
        store_px_planar<FMT, TE>(a.out_col, idx, col, tab + 256);
        if (a.out_blackout) store_px_planar<FMT, TE>(a.out_blackout, idx, bo, tab + 256);
        const uint64_t m = __builtin_amdgcn_ballot_w64(zero);
        if ((uint32_t)(idx & 63u) == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec())) {
            const size_t w = ((idx >> 6) * TE + 192u) * CB / 8u;  // the mask word (8-byte aligned)
            reinterpret_cast<uint64_t*>(a.out_col)[w] = m;
            if (a.out_blackout) reinterpret_cast<uint64_t*>(a.out_blackout)[w] = m;
        }
    } else if (a.layout == BH_LAYOUT_TILES_RGBM14) {
        if constexpr (FMT == BH_OUT_RGBA16F) {  // bh_render admits this layout for RGBA16F only
            store_rgbm14(a.out_col, idx, col, zero);
            if (a.out_blackout) store_rgbm14(a.out_blackout, idx, bo, zero);
        }
    } else {
        store_px<FMT>(a.out_col, idx, col, tab + 256);
        if (a.out_blackout) store_px<FMT>(a.out_blackout, idx, bo, tab + 256);
    }
    if (a.dbg_n_rk) a.dbg_n_rk[idx] = (uint16_t)n_rk;
    if (a.dbg_fate) a.dbg_fate[idx] = (uint8_t)fate;
    if (a.dbg_steps) a.dbg_steps[idx] = (uint16_t)steps;
}
template <uint32_t FMT>
__device__ __forceinline__ void write_pixel(const MarchArgs& a, const float* tab, size_t idx, v3 col, uint32_t n_rk,
                                            uint32_t fate) {
    write_pixel<FMT>(a, tab, idx, col, n_rk, fate, n_rk);
}

// 32-bit pixel index: width, height <= 65536 (bh_render), so py * W + px < 2^32; a shard holds < 2^24 tiles
__device__ __forceinline__ uint32_t out_index(const MarchArgs& a, uint32_t t, uint32_t lane, uint32_t px, uint32_t py) {
    return (a.layout != BH_LAYOUT_ROWMAJOR) ? t * 64u + lane : py * a.width + px;
}

// Iterations after which a still-marching wave raises its issue priority (the frame's tail: measured
// +34 % of kernel time at cap 512 vs cap 64 without it) and the tile schedule starts checking for
// cycles (march_cycles).
constexpr uint32_t PRIO_ITERS = 48;

// Waves per workgroup of the tile schedule.  One: a workgroup's LDS (1 KiB decode table + 4 KiB
// cycle history) is released when its one wave ends, and a new wave needs no three other free
// slots on the CU; no workgroup barrier beyond the wave's own table load.  1 vs 4 waves (interleaved
// A/B, profiles/r02d/ab_wg/): headline -0.6 %, 1920x1080 -0.8 %, cap 1000 -1.0 %, one frame per
// launch -1.4 %, 256x256 cap 64 +0.6 % (noise level).  32 such workgroups per CU fill its 160 KiB.
constexpr uint32_t WG_WAVES = 1u;

// ---- schedule BH_SCHED_TILE: one wave64 = one 8x8 tile (default) ---------------------------------
// Dispatch slot -> tile through `order` (previous frame's per-tile cost, expensive tiles first) or
// the centre-out permutation; each wave records its tile's max n_rk for the next frame's order.
// wave_max_u32: bh_common.hpp

// ---- cycle fast-forward ----------------------------------------------------------------------------
// One loop iteration is a pure function of (ro, rd, travelled, outside) (s and the uniforms are
// per-ray constants; n_rk only feeds the cap test).  Some rays stop moving in f32: dt rounds to 0 on
// the photon-sphere marker (dps == 0 exactly, a fixed point) or flips sign every step around it (a
// 2-cycle); they then iterate unchanged until the cap (SURVEY §8d "Zeno" rays, up to 512 steps).
// After step j, if the state equals the state two steps back bit for bit (and `outside` did not
// change across those two steps), the sequence is periodic with period 1 or 2 from then on; no
// termination test can fire (both states of the cycle already passed them), so the ray ends with
// fate CAP, n_rk = max_iters and the cycle state of matching parity: the loop's own result,
// without running it.  Checked from PRIO_ITERS on (the cycles found start at median iteration 30).
struct Hist { v3 ro, rd; float tr; uint32_t outside; };

__device__ __forceinline__ bool same_bits(float x, float y) { return __float_as_uint(x) == __float_as_uint(y); }
__device__ __forceinline__ bool same_state(const RayState& st, const Hist& h) {
    // bitwise & (no short-circuit branches)
    return same_bits(st.ro.x, h.ro.x) & same_bits(st.ro.y, h.ro.y) & same_bits(st.ro.z, h.ro.z) &
           same_bits(st.rd.x, h.rd.x) & same_bits(st.rd.y, h.rd.y) & same_bits(st.rd.z, h.rd.z) &
           same_bits(st.travelled, h.tr) & (st.outside == h.outside);
}

// March `st` to termination with the fast-forward; `steps` = RK updates actually executed.  The two
// history states live in LDS (ping-pong slots by iteration parity), not VGPRs: holding them in
// registers takes the kernel from 61 to 73 VGPRs (8 -> 6 waves per SIMD) and measured slower.
struct HistLds { float4 a[2][2][64]; };  // [slot][ro+tr | rd+outside][lane]
// XOR-fold of the state compared by same_state: equal states have equal hashes, so a hash match is
// only a candidate and the full states (in LDS) decide.  The hashes live in 2 VGPRs, so the common
// case reads no LDS and never waits for it (the serial chain of a lone tail wave is the frame's
// critical path).
__device__ __forceinline__ uint32_t state_hash(const RayState& st) {
    return (__float_as_uint(st.ro.x) ^ __float_as_uint(st.ro.y) ^ __float_as_uint(st.ro.z) ^
            __float_as_uint(st.rd.x) ^ __float_as_uint(st.rd.y) ^ __float_as_uint(st.rd.z) ^
            __float_as_uint(st.travelled)) + st.outside * 0x9E3779B9u;
}
// The workgroup's history areas (4 KiB per wave: 8 waves per SIMD still fit, 5 KiB x 32).
template <int>
__device__ __forceinline__ HistLds* hist_lds() {
    __shared__ HistLds hist[WG_WAVES];
    return hist;
}

// March `st` to termination with the fast-forward; `steps` = RK updates actually executed.
// (The tail waves are latency-bound: a ping-pong / uniform-trip form of this loop measured slower.)
// Cycles are looked for until iteration CYCLE_ITERS_END only: the ones found start by iteration ~50
// (median 30); the rays still marching after that crawl or orbit without repeating, and
// stopping the search never changes a result -- the loop then just runs to its normative end.
constexpr uint32_t CYCLE_ITERS_END = 192u;
template <uint32_t SF>
__device__ __forceinline__ uint32_t march_cycles(const MarchArgs& a, const Frame& f, RayState& st, uint32_t& steps,
                                                 HistLds& H, uint32_t lane) {
    // h2: hash of the state two iterations back (none yet: a value that forces a full compare
    // against slot 1, whose travelled is a NaN pattern no arithmetic produces -- no match)
    H.a[1][0][lane] = make_float4(st.ro.x, st.ro.y, st.ro.z, __uint_as_float(0xFFFFFFFFu));
    H.a[1][1][lane] = make_float4(st.rd.x, st.rd.y, st.rd.z, __uint_as_float(st.outside));
    uint32_t h2 = ~state_hash(st), h1 = 0;
    for (uint32_t p = 0;; p ^= 1u) {
        H.a[p][0][lane] = make_float4(st.ro.x, st.ro.y, st.ro.z, st.travelled);
        H.a[p][1][lane] = make_float4(st.rd.x, st.rd.y, st.rd.z, __uint_as_float(st.outside));
        h1 = state_hash(st);
        const uint32_t fate = march_step_tail<SF>(a, f, st);
        if (fate != 0xFFu) { steps = st.n_rk; return fate; }
        if (st.n_rk >= CYCLE_ITERS_END) break;  // wave-uniform: every live lane is at the same iteration
        if (state_hash(st) == h2) {
            const float4 q0 = H.a[p ^ 1u][0][lane], q1 = H.a[p ^ 1u][1][lane];
            const Hist hs{mk(q0.x, q0.y, q0.z), mk(q1.x, q1.y, q1.z), q0.w, __float_as_uint(q1.w)};
            if (same_state(st, hs)) {
                steps = st.n_rk;
                if ((a.max_iters - st.n_rk) & 1u) {
                    const float4 r0 = H.a[p][0][lane], r1 = H.a[p][1][lane];
                    st.ro = mk(r0.x, r0.y, r0.z); st.rd = mk(r1.x, r1.y, r1.z); st.travelled = r0.w;
                }
                st.n_rk = a.max_iters;
                return BH_FATE_CAP;
            }
        }
        h2 = h1;
    }
    // past CYCLE_ITERS_END: the plain loop, no history writes or hashes (a lone tail wave's step is
    // issue-bound, and those were ~8 % of its instructions)
    for (;;) {
        const uint32_t fate = march_step_tail<SF>(a, f, st);
        if (fate != 0xFFu) { steps = st.n_rk; return fate; }
    }
}

// The per-frame fields of frame f of a multi-frame launch: its camera (read before and in the march
// loop) and its outputs (read after it).
__device__ __forceinline__ void select_camera(MarchArgs& a, const FrameArgs& F) {
    for (int k = 0; k < 3; ++k) {
        a.pos[k] = F.pos[k]; a.c0[k] = F.c0[k]; a.c1[k] = F.c1[k]; a.c2[k] = F.c2[k]; a.cps[k] = F.cps[k];
    }
}
__device__ __forceinline__ void select_outputs(MarchArgs& a, const FrameArgs& F) {
    a.out_col = F.out_col; a.out_blackout = F.out_blackout;
    a.dbg_n_rk = F.dbg_n_rk; a.dbg_fate = F.dbg_fate; a.dbg_steps = F.dbg_steps;
}

// March one ray to its end (the tile schedule's loop): `fate` and `steps` (RK updates executed).
template <uint32_t SF>
__device__ __forceinline__ void march_ray(const MarchArgs& a, const Frame& f, RayState& st, uint32_t& fate,
                                          uint32_t& steps, uint32_t lane) {
    // Two iterations per trip, ping-ponging the state between st and sb (march_step_io never
    // writes its input, so no per-step register copies).  The lane's final state is the output
    // of its last iteration, or its input for the fates decided before the RK update: the one of
    // st / sb with the larger n_rk, once a lane leaving before the RK update has zeroed the
    // other's n_rk (it may hold a discarded output of the guarded first pass).  The input of
    // iteration i holds n_rk = i and the other register i - 1 or (i = 0) the same state, so no
    // per-step flag records where the state is (-6 VALU per step: headline -0.5 %, A/B r02,
    // profiles/r02c/ab_inb/).  The trip condition is wave-uniform and each lane's iteration is
    // predicated: with a divergent loop exit the state would be live out of the loop at a
    // different iteration per lane, which costs a register copy of every state value per
    // iteration.  (390 -> 370 VALU per step; with the flag template and the guard pooling
    // 0.842 -> 0.837 ms headline, 0.99 -> 0.92 ms at cap 1000, A/B r01.)
    RayState sb = st;
    bool alive = true;
    // TRIP_PAIRS ping-pong pairs per trip of the wave-uniform loop (1 / 2 / 3 pairs: 0.689 / 0.688
    // / 0.686 ms, A/B r01): fewer trip tests and their ballot materialisation per step.
    constexpr uint32_t TRIP_PAIRS = 3;
    static_assert(PRIO_ITERS % (2u * TRIP_PAIRS) == 0u, "whole trips");
    for (uint32_t it = 0; it < PRIO_ITERS && __builtin_amdgcn_ballot_w64(alive) != 0ull; it += 2u * TRIP_PAIRS) {
#pragma unroll
        for (uint32_t j = 0; j < TRIP_PAIRS; ++j) {
            if (alive) {
                if (march_step_io<SF, true>(a, f, st, sb, fate, it + 2u * j)) {
                    alive = false;
                    if (fate_before_rk(fate)) sb.n_rk = 0u;
                }
            }
            if (alive) {
                if (march_step_io<SF, true>(a, f, sb, st, fate, it + 2u * j + 1u)) {
                    alive = false;
                    if (fate_before_rk(fate)) st.n_rk = 0u;
                }
            }
        }
    }
    if (sb.n_rk > st.n_rk) st = sb;
    steps = st.n_rk;
    if (alive) {
        // A wave still marching after PRIO_ITERS iterations (~4x the mean step count) holds a
        // photon-sphere ray that may run to the cap: raise its issue priority so its serial chain
        // is not stretched by the SIMD's other waves (the frame's tail), and watch for cycles.
        __builtin_amdgcn_s_setprio(2);
        fate = march_cycles<SF>(a, f, st, steps, hist_lds<0>()[threadIdx.x >> 6], lane);
    }
}

// Several frames in one launch (bh_render_frames): dispatch slot s is tile s / n_frames of the order
// in frame s % n_frames, so every frame's expensive tiles start first and one frame's serial tail
// overlaps the others' bulk instead of ending the launch alone.  Only frame 0
// records the tile costs for the next launch's order (the histogram must count each tile once).
//

// One dispatch slot, marched by one wave.
template <uint32_t FMT, uint32_t SF>
__device__ __forceinline__ void march_slot(const MarchArgs& A, uint32_t slot, const float* lut,
                                           uint32_t lane) {
    const uint32_t nf = A.n_frames;
    uint32_t fi = 0, j = slot;
    if (nf > 1u) {
        j = slot / nf;
        fi = slot - j * nf;
    }
    MarchArgs a = A;
    // frames[0] == the top-level fields for a one-frame launch; launches of more than
    // BH_INLINE_FRAMES frames read them from the device table (wave-uniform index: one load per wave)
    if (A.frame_table) select_camera(a, A.frame_table[fi]);
    else select_camera(a, A.frames[fi]);
    if (fi != 0u) a.tile_cost = nullptr;
    const uint32_t t = a.order ? a.order[j] : centre_out(j, a.n_tiles, a.order_block, a.order_centre);
    if (t >= a.n_tiles) return;  // defensive: a corrupt order must not address outside the shard
    uint32_t tx, ty;
    if (a.tile_list) {  // weighted partition (bh_partition): the shard's tile list
        const uint32_t v = a.tile_list[t];
        tx = v & 0xFFFFu;
        ty = v >> 16;
    } else {
        shard_tile_coords(t, a.tiles_x, a.shard_index, a.shard_count, &tx, &ty);
    }
    const uint32_t px = tx * 8u + (lane & 7u), py = ty * 8u + (lane >> 3);
    const bool valid = px < a.width && py < a.height;
    const Frame f = make_frame(a);
    RayState st;
    st.ro = f.ro0;
    st.rd = pixel_ray(a, valid ? px : 0u, valid ? py : 0u);
    st.s = ray_s(f, st.rd);
    st.travelled = 0.0f;
    st.n_rk = 0;
    st.outside = 0u;
    uint32_t fate = 0xFFu, steps = 0;
    if (valid) {
        // the camera outside the unit sphere (1.01 leaves room for any rounding of |ro0|^2 against the
        // step's own r^2 > 1 + 2^-23 at iteration 0) and |s| <= 2^30 on every lane: the step without the
        // ingoing test and the |s| guard (wave-uniform: a scalar branch)
        if constexpr (SF != SF_DYN) {
            const bool out = (dot(f.ro0, f.ro0) > 1.01f) && (__builtin_amdgcn_ballot_w64(!(fabsf(st.s) <= 0x1p30f)) == 0ull);
            if (__builtin_amdgcn_readfirstlane((int)out)) march_ray<SF | SF_CAM_OUT>(a, f, st, fate, steps, lane);
            else march_ray<SF>(a, f, st, fate, steps, lane);
        } else {
            march_ray<SF>(a, f, st, fate, steps, lane);
        }
    }
    if (valid) {
        // the frame's output pointers are loaded here, from an opaque copy of the frame index: loaded
        // up front they would hold 10 SGPRs through the march loop, over the 80 that keep 8
        // workgroups per CU resident (MI355X_MICROARCH.md, Residency)
        uint32_t fo = fi;
        asm volatile("" : "+s"(fo));
        if (A.frame_table) select_outputs(a, A.frame_table[fo]);
        else select_outputs(a, A.frames[fo]);
#if BH_SKY_LDS && !BH_FAST
        const v3 col = shade_tile(a, lut, fate, st.rd, reinterpret_cast<uint32_t*>(&hist_lds<0>()[threadIdx.x >> 6]), lane);
#else
        const v3 col = shade(a, lut, fate, st.rd);
#endif
        write_pixel<FMT>(a, lut, out_index(a, t, lane, px, py), col, st.n_rk, fate, steps);
    }
    if (a.tile_cost) {
        // the next frame's cost and its bucket histogram (a no-return atomic: the wave does not wait);
        // the last bucket is the remainder and is not counted
        const uint32_t m = min(wave_max_u32(steps) >> 1, 255u);
        if (lane == 0u) {
            a.tile_cost[t] = (uint8_t)m;
            const uint32_t b = cost_bucket(m);
            if (b < ORDER_BUCKETS - 1u)
                __hip_atomic_fetch_add(&a.order_tot[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Shader-clock probe (bh_set_clock_probe): a sampled wave reads both counters when it starts and adds
// the differences at its end to its XCD's accumulators (vector atomics from lane 0, no return).  (A
// divergent lane-0 branch before the march trips an "illegal VGPR to SGPR copy" in this compiler, so
// the start values are held in 2 SGPRs instead: their low 32 bits, since a wave lives far less than
// 2^32 shader cycles.)
struct ClockStart { uint32_t t, r; };
__device__ __forceinline__ ClockStart clock_start() {
    return {(uint32_t)__builtin_amdgcn_s_memtime(), (uint32_t)__builtin_amdgcn_s_memrealtime()};
}
__device__ __forceinline__ void clock_end(unsigned long long* acc, const ClockStart& c0) {
    const uint32_t t = (uint32_t)__builtin_amdgcn_s_memtime() - c0.t;      // shader clock
    const uint32_t r = (uint32_t)__builtin_amdgcn_s_memrealtime() - c0.r;  // constant 100 MHz
    const uint32_t x = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;  // HW_REG_XCC_ID[2:0]
    // a sample whose ratio is outside 0.5-4 GHz is dropped: a wave saved and restored elsewhere (queue
    // preemption) reads another XCD's shader counter at its end (seen once: 20 GHz on two XCDs)
    const bool sane = (uint64_t)t >= 5ull * r && (uint64_t)t <= 40ull * r;
    if ((threadIdx.x & 63u) == 0u && sane) {
        unsigned long long* p = acc + 16u * x;
        __hip_atomic_fetch_add(p, (unsigned long long)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(p + 1, (unsigned long long)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(p + 2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// One wave per dispatch slot (the grid covers every slot), WG_WAVES waves per workgroup.
template <uint32_t FMT, uint32_t SF>
__global__ void __launch_bounds__(64 * WG_WAVES) march_tile_kernel(MarchArgs A) {
    __shared__ float lut[lds_tables<FMT>()];
    load_tables<FMT, 64u * WG_WAVES>(A, lut);
    __syncthreads();
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * WG_WAVES + (threadIdx.x >> 6));
    const uint32_t n_slots = A.n_tiles * A.n_frames;
    {
        const uint32_t slot = w;
        if (slot >= n_slots) return;  // wave-uniform
        // one slot in `stride`, rotated by slot / stride: the dispatcher deals workgroups to the 8 XCDs
        // round robin, so plain multiples of the stride would all land on one XCD
        const bool probe = A.clk && ((slot + (slot >> 8)) & A.clk_mask) == 0u;
        ClockStart c0{0u, 0u};
        if (probe) c0 = clock_start();
        march_slot<FMT, SF>(A, slot, lut, threadIdx.x & 63u);
        if (probe) clock_end(A.clk, c0);
    }
}

// ---- schedule BH_SCHED_PERSISTENT: persistent waves with per-lane refill (A/B option) ------------
//
// Each wave keeps all 64 lanes marching.  Rays are prepared (pixel_ray + s, :362-363, :262-263) in
// full-width batches of one 8x8 tile into an LDS "ready" queue, and a lane whose ray terminates pops
// the next ready ray at once, so no lane idles while a slow (photon-sphere "Zeno", capped) ray runs
// on.  Finished rays are pushed into an LDS "done" queue and shaded (sky lookup, :329-345) in
// full-width batches of 64.  Tiles are dequeued from NQ work counters (one 128-B line each; the
// shard-local tile range is split into NQ contiguous parts; a wave starts on part blockIdx % NQ and
// moves on when it is exhausted), so the result never depends on dispatch order or placement.
constexpr uint32_t NQ = 8;
constexpr uint32_t CTR_STRIDE = 32;  // u32 words between counters (128 B)
constexpr uint32_t READY_CAP = 128;
constexpr uint32_t DONE_CAP = 128;

struct WaveQueues {
    float r_x[READY_CAP], r_y[READY_CAP], r_z[READY_CAP], r_s[READY_CAP];
    uint32_t r_idx[READY_CAP];
    float d_x[DONE_CAP], d_y[DONE_CAP], d_z[DONE_CAP];
    uint32_t d_idx[DONE_CAP], d_meta[DONE_CAP];  // meta = fate << 16 | n_rk
};

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {  // set lanes below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <uint32_t FMT>
__global__ void __launch_bounds__(256) march_persistent_kernel(MarchArgs a, uint32_t* __restrict__ counters) {
    __shared__ float lut[lds_tables<FMT>()];
    __shared__ WaveQueues queues[4];
    load_tables<FMT>(a, lut);
    __syncthreads();  // the only workgroup barrier: waves run independently afterwards

    const uint32_t lane = threadIdx.x & 63u;
    WaveQueues& Q = queues[threadIdx.x >> 6];
    const Frame f = make_frame(a);
    const uint32_t T = a.n_tiles;

    uint32_t part = blockIdx.x % NQ, parts_left = NQ;  // work-queue cursor (wave-uniform)
    uint32_t n_ready = 0, n_done = 0;                  // queue fill levels (wave-uniform)

    RayState st;
    st.ro = f.ro0; st.rd = f.ro0; st.s = 0.0f; st.travelled = 0.0f; st.n_rk = 0; st.outside = 0u;
    uint32_t idx = 0;
    bool alive = false;

    for (;;) {
        // -- refill dead lanes from the ready queue; top the queue up with one tile if short --
        const uint64_t dead = __ballot(!alive);
        const uint32_t n_dead = __popcll(dead);
        if (n_dead != 0u) {
            while (n_ready < n_dead && parts_left != 0u) {
                // dequeue one tile
                uint32_t t = 0xFFFFFFFFu;
                if (lane == 0) {
                    const uint32_t lo = (uint32_t)((uint64_t)T * part / NQ);
                    const uint32_t hi = (uint32_t)((uint64_t)T * (part + 1u) / NQ);
                    const uint32_t i = atomicAdd(&counters[part * CTR_STRIDE], 1u);
                    t = (lo + i < hi) ? lo + i : 0xFFFFFFFFu;
                }
                t = __builtin_amdgcn_readfirstlane(t);
                if (t == 0xFFFFFFFFu) { part = (part + 1u) % NQ; --parts_left; continue; }
                uint32_t tx, ty;
                shard_tile_coords(t, a.tiles_x, a.shard_index, a.shard_count, &tx, &ty);
                const uint32_t px = tx * 8u + (lane & 7u), py = ty * 8u + (lane >> 3);
                const bool valid = px < a.width && py < a.height;
                const uint64_t vm = __ballot(valid);
                if (valid) {
                    const v3 rd0 = pixel_ray(a, px, py);
                    const uint32_t e = n_ready + lane_rank(vm);
                    Q.r_x[e] = rd0.x; Q.r_y[e] = rd0.y; Q.r_z[e] = rd0.z;
                    Q.r_s[e] = ray_s(f, rd0);
                    Q.r_idx[e] = (uint32_t)out_index(a, t, lane, px, py);
                }
                n_ready += (uint32_t)__popcll(vm);
            }
            __builtin_amdgcn_wave_barrier();
            if (n_ready != 0u) {
                if (!alive) {
                    const uint32_t k = lane_rank(dead);
                    if (k < n_ready) {
                        const uint32_t e = n_ready - 1u - k;
                        st.ro = f.ro0;
                        st.rd = mk(Q.r_x[e], Q.r_y[e], Q.r_z[e]);
                        st.s = Q.r_s[e];
                        idx = Q.r_idx[e];
                        st.travelled = 0.0f; st.n_rk = 0; st.outside = 0u;
                        alive = true;
                    }
                }
                n_ready -= (n_dead < n_ready) ? n_dead : n_ready;
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (__ballot(alive) == 0ull) break;  // no rays left anywhere for this wave

        // -- one RK iteration for every live lane --
        uint32_t fate = 0xFFu;
        if (alive) fate = march_step(a, f, st);
        const bool fin = fate != 0xFFu;
        const uint64_t fm = __ballot(fin);
        if (fm != 0ull) {
            if (fin) {
                const uint32_t e = n_done + lane_rank(fm);
                Q.d_x[e] = st.rd.x; Q.d_y[e] = st.rd.y; Q.d_z[e] = st.rd.z;
                Q.d_idx[e] = idx;
                Q.d_meta[e] = (fate << 16) | st.n_rk;
                alive = false;
            }
            n_done += (uint32_t)__popcll(fm);
            __builtin_amdgcn_wave_barrier();
            // -- shade a full batch of 64 finished rays --
            if (n_done >= 64u) {
                const uint32_t e = n_done - 64u + lane;
                const uint32_t meta = Q.d_meta[e];
                const v3 col = shade(a, lut, meta >> 16, mk(Q.d_x[e], Q.d_y[e], Q.d_z[e]));
                write_pixel<FMT>(a, lut, Q.d_idx[e], col, meta & 0xFFFFu, meta >> 16);
                n_done -= 64u;
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
    // -- shade what is left --
    if (lane < n_done) {
        const uint32_t meta = Q.d_meta[lane];
        const v3 col = shade(a, lut, meta >> 16, mk(Q.d_x[lane], Q.d_y[lane], Q.d_z[lane]));
        write_pixel<FMT>(a, lut, Q.d_idx[lane], col, meta & 0xFFFFu, meta >> 16);
    }
}

// ---- schedule BH_SCHED_PAIR: two rays per lane (A/B option) --------------------------------------
// One wave64 = two consecutive shard-local 8x8 tiles; each lane marches the pixel at the same (x&7,
// y&7) position in both (8 px apart for an unsharded frame: coherent step counts) and the loop body
// interleaves the two rays' iterations: on gfx950 one dependent chain per wave issues only every
// ~4-5 cycles however many waves share the SIMD, two chains reach the ~2.3-cycle peak
// (tools/ubench/latency.hip).  Measured slower than the tile schedule (113 VGPRs: 4 waves per
// SIMD instead of 8).
template <uint32_t FMT>
__global__ void __launch_bounds__(256) march_pair_kernel(MarchArgs a) {
    __shared__ float lut[lds_tables<FMT>()];
    load_tables<FMT>(a, lut);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t pair = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t npairs = (a.n_tiles + 1u) / 2u;
    if (pair >= npairs) return;
    // centre-out over pairs (block = half a tile row of pairs); tiles 2p, 2p+1 stay adjacent
    const uint32_t pp = centre_out(pair, a.n_tiles / 2u, a.order_block / 2u, a.order_centre);
    const uint32_t t0 = 2u * pp, t1 = t0 + 1u;
    const Frame f = make_frame(a);
    uint32_t px0 = 0, py0 = 0, px1 = 0, py1 = 0;
    {
        uint32_t tx, ty;
        shard_tile_coords(t0, a.tiles_x, a.shard_index, a.shard_count, &tx, &ty);
        px0 = tx * 8u + (lane & 7u); py0 = ty * 8u + (lane >> 3);
        if (t1 < a.n_tiles) {
            shard_tile_coords(t1, a.tiles_x, a.shard_index, a.shard_count, &tx, &ty);
            px1 = tx * 8u + (lane & 7u); py1 = ty * 8u + (lane >> 3);
        }
    }
    bool alive0 = px0 < a.width && py0 < a.height;
    bool alive1 = t1 < a.n_tiles && px1 < a.width && py1 < a.height;
    const bool valid0 = alive0, valid1 = alive1;
    RayState s0, s1;
    s0.ro = f.ro0; s0.travelled = 0.0f; s0.n_rk = 0; s0.outside = 0u;
    s1 = s0;
    s0.rd = sel(valid0, pixel_ray(a, px0, py0), f.ro0);
    s1.rd = sel(valid1, pixel_ray(a, px1, py1), f.ro0);
    s0.s = ray_s(f, s0.rd);
    s1.s = ray_s(f, s1.rd);
    uint32_t fate0 = BH_FATE_CAP, fate1 = BH_FATE_CAP;
    for (uint32_t it = 0; alive0 || alive1; ++it) {
        if (it == PRIO_ITERS) __builtin_amdgcn_s_setprio(2);
        march_step2(a, f, s0, s1, alive0, alive1, fate0, fate1);
    }
    if (valid0) write_pixel<FMT>(a, lut, out_index(a, t0, lane, px0, py0), shade(a, lut, fate0, s0.rd), s0.n_rk, fate0);
    if (valid1) write_pixel<FMT>(a, lut, out_index(a, t1, lane, px1, py1), shade(a, lut, fate1, s1.rd), s1.n_rk, fate1);
}

// Host side: launch the tile schedule, one wave per dispatch slot.  (A persistent form -- resident
// waves claiming slots in order from one device-scope counter -- measured 2.5x slower: a returning
// atomic on one word is serialised across the 8 XCDs at ~85 M claims/s)
template <uint32_t FMT, uint32_t SF>
inline void launch_tile_schedule(const MarchArgs& a, hipStream_t s) {
    const uint32_t waves = a.n_tiles * a.n_frames;
    const uint32_t blocks = (waves + (WG_WAVES - 1u)) / WG_WAVES;
    hipLaunchKernelGGL((march_tile_kernel<FMT, SF>), dim3(blocks), dim3(64u * WG_WAVES), 0, s, a);
}

}  // namespace BH_NS
}  // namespace bh
