// bh_crmath.hpp — correctly rounded f32 division and square root for gfx950, cheap forms.
//
// hipcc's IEEE division expands to 11 VALU ops (v_div_scale x2, v_rcp, 6 FMA-class ops, v_div_fmas,
// v_div_fixup) and measures ~50 cycles per wave-instruction stream on MI355X; its IEEE sqrt ~54
// (tools/ubench/valu_rates.hip).  The march loop needs 18 divisions and 7 square roots per RK step,
// so these dominate the exact (bit-parity) kernel.  The forms below drop the scaling/fix-up steps,
// which only act on operands near the ends of the exponent range, share one correctly rounded
// reciprocal between the three divisions of rd_derivative, and are as short as exhaustive checks
// on the device allow (tools/ubench/cr_forms.hip).  Each form is the SAME arithmetic as hipcc's
// correctly-rounded expansion inside its safe domain, and each caller accumulates a "bad" flag for
// operands outside that domain; the march loop then redoes that RK step with plain IEEE ops
// (bh_march.hpp, march_step).  tests/test_gpu_crmath.py checks every form against IEEE results on
// ~10^9 inputs per form on the GPU (bh_selftest_crmath), including the boundaries.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {
namespace crm {

// ---- square root ------------------------------------------------------------------------------
// One Newton step on the hardware reciprocal square root: y = v_rsq(x), s = x*y, and the residual
// x - s*s (exact in an FMA) corrects s by y/2:  sqrt(x) = fma(x - s*s, y/2, s).  1 transcendental + 4
// VALU ops (the previous form, v_sqrt + a residual test of both neighbours, took 1 + 8).  Equal to
// the IEEE sqrt for EVERY float x in [2^-102, FLT_MAX] (exhaustive, tools/ubench/cr_forms.hip on
// MI355X; profiles/r01_cr_forms.log); wrong for 0 (0*inf), +inf (inf*0) and x < 2^-102, so the guard
// is the range [SQRT_MIN, FLT_MAX] (NaN fails it too).
constexpr float SQRT_MIN = 0x1p-96f;
constexpr float SQRT_MAX = 0x1.fffffep127f;

__device__ __forceinline__ float sqrt_core(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y;
    const float h = 0.5f * y;
    const float r = __builtin_fmaf(-s, s, x);
    return __builtin_fmaf(r, h, s);
}
// the same, also handing back the v_rsq estimate y it refined (rcp_from_rsq seeds a reciprocal from it)
struct SqrtY { float s, y; };
__device__ __forceinline__ SqrtY sqrt_core_y(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y;
    const float h = 0.5f * y;
    const float r = __builtin_fmaf(-s, s, x);
    return {__builtin_fmaf(r, h, s), y};
}
// unsafe iff x is outside [2^-96, FLT_MAX] (0, +inf and NaN included)
__device__ __forceinline__ bool sqrt_bad(float x) { return !(x >= SQRT_MIN && x <= SQRT_MAX); }
// the same for two values (one v_min + one v_max + two compares)
__device__ __forceinline__ bool sqrt_bad2(float a, float b) {
    return !(fminf(a, b) >= SQRT_MIN) | !(fmaxf(a, b) <= SQRT_MAX);
}

// ---- division by a shared denominator ---------------------------------------------------------
// r = v_rcp(d) refined once, r += r*(1 - d*r), is the correctly rounded reciprocal RN(1/d) for every
// normal d whose reciprocal is normal (exhaustive on MI355X, tools/ubench/cr_forms.hip op R).  Then
// y = n*r and ONE residual correction  q = y + r*(n - d*y)  is RN(n/d) (Markstein's theorem; checked
// exhaustively over all 2^46 pairs of significands n, d in [1, 2) against the two-correction
// sequence of hipcc's IEEE division, op D; every op is exactly scale-covariant in the guarded normal
// range, op X, so the square covers the domain).  Domain (the caller guarantees it):
//   DIV_D_MIN <= d <= DIV_D_MAX  (checked per denominator, div_d_bad)
//   n == 0 or DIV_N_MIN <= |n| <= 2^64
// The residual is formed negated, e = d*y - n = -(n - d*y) (exact in an FMA, RN is symmetric), and
// added back as fma(-e, r, y): identical for n != 0, and for n = +-0 the sum keeps the IEEE sign of
// the zero quotient (-0 + -0 = -0) without a copysign.
constexpr float DIV_D_MIN = 0x1p-40f;
constexpr float DIV_D_MAX = 0x1p+60f;
constexpr float DIV_N_MIN = 0x1p-60f;

struct Rcp { float d, r; };

__device__ __forceinline__ Rcp rcp_refined(float d) {
    float r = __builtin_amdgcn_rcpf(d);
    const float e = __builtin_fmaf(-d, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    return {d, r};
}
// RN(1/Q) of rd_derivative's denominator Q = RN(RN(q*q) * sqrt(q)) without a second transcendental:
// y = v_rsq(q) (the square-root core's own estimate) gives the seed z = (y^2)^2 * y ~ q^-2.5 (three
// multiplies, 6 issue cycles, where v_rcp takes 8 and blocks the SIMD's vector issue for all of them:
// tools/ubench/trans_mix.hip), within ~2^-20 of 1/Q; one refinement r = z + z(1 - Qz) lands within
// ~2^-40 of 1/Q before its rounding: RN(1/Q) except where 1/Q lies within that of a rounding midpoint (840
// of the 3.5e8 q in [2^-17, 2^25), selftest op 12), where it is the faithful neighbour -- and with that
// neighbour div_core's one correction misses the IEEE quotient for 60 (n, Q) pairs, at Q significands
// next to 2 (selftest op 13).  So the march keeps rcp_refined (BH_RCP_SEED 0); measured, not used.
__device__ __forceinline__ Rcp rcp_from_rsq(float Q, float y) {
    const float y2 = y * y, y4 = y2 * y2, z = y4 * y;
    const float e = __builtin_fmaf(-Q, z, 1.0f);
    return {Q, __builtin_fmaf(e, z, z)};
}
__device__ __forceinline__ float div_core(float n, const Rcp& R) {
    const float y = n * R.r;
    const float e = __builtin_fmaf(R.d, y, -n);
    return __builtin_fmaf(-e, R.r, y);
}
__device__ __forceinline__ bool div_d_bad(float d) { return !(d >= DIV_D_MIN && d <= DIV_D_MAX); }

// ---- division by 6 and by 12 ------------------------------------------------------------------
// 1/D split as H + L: H = RD_f32(1/D), L = RN_f32(1/D - H) > 0.  x/D = fma(x, H, x*L) rounds
// x*H + RN(x*L) once; that sum is within 2^-47 relative of x/D, while x/D (x a 24-bit significand over
// 3 * 2^k) is either exact or at least 1/6 ulp away from every rounding midpoint, so the one rounding
// is RN(x/D).  Two ops instead of the three of y = x*RN(1/D) plus a residual correction.  Both terms
// carry x's sign (H, L > 0), so x = +-0 gives the IEEE zero.  Exhaustive: equal to IEEE x/6 and
// x/12 for every finite x with |x| >= 2^-121 and for +-0 (x*L loses bits below that); the callers'
// domain is x == 0 or |x| >= DIV_N_MIN (selftest ops 1 and 5 on the GPU over all 2^32 patterns,
// tools/ubench/div_const.c on the host).
constexpr float R6_H = 0x1.555554p-3f, R6_L = 0x1.555556p-27f;
constexpr float R12_H = 0x1.555554p-4f, R12_L = 0x1.555556p-28f;
__device__ __forceinline__ float div6(float x) { return __builtin_fmaf(x, R6_H, x * R6_L); }
__device__ __forceinline__ float div12(float x) { return __builtin_fmaf(x, R12_H, x * R12_L); }

// key(n) = 2*bits(|n|) - 1 (mod 2^32): +-0 -> 0xFFFFFFFF, tiny -> small, so key(n) < KEY_MIN iff
// 0 < |n| < DIV_N_MIN; a running v_min3_u32 over keys needs one compare per step.  (A float
// min of |n| would be one op cheaper but cannot tell 0 from tiny: measured 2x slower overall,
// because every camera-A ray starts on two coordinate planes and its first step then re-runs.)
constexpr uint32_t KEY_MIN = (0x21800000u << 1) - 1u;  // key(2^-60)
// The march's acceleration numerators s * p_i are held to the stricter 0 or >= 2^-40 (ACC_N_MIN): then
// every acceleration component is 0 or >= 2^-100 (Q <= 2^60), which the fma form of the RK stage
// directions relies on (bh_march.hpp, XOps::rd_half).  Still inside the division core's domain.
constexpr float ACC_N_MIN = 0x1p-40f;
constexpr uint32_t KEY_ACC_MIN = (0x2B800000u << 1) - 1u;  // key(2^-40)
__device__ __forceinline__ uint32_t key(float n) { return (__float_as_uint(n) << 1) - 1u; }
__device__ __forceinline__ uint32_t kmin3(uint32_t a, uint32_t b, uint32_t c) { return min(min(a, b), c); }


// ---- atan2 rounded to f32 ----------------------------------------------------------------------
// The normative shading angle is RN_f32(atan2(y, x)) evaluated in f64 (the oracle calls
// the C library's f64 atan2, the first kernels ocml's).  atan2_core computes the f64 angle A in fewer
// and cheaper operations than ocml's general f64 atan2 (whose IEEE division and degree-20 polynomial
// with 64-bit literal coefficients took ~110 instructions per wave): octant reduction to
// u = mn / mx, or (mn - mx) / (mn + mx) when mn / mx > tan(pi/8) (both exact in f64 for f32
// inputs: the exponents are within 2 there), a reciprocal refined twice and one residual correction
// (RN-accurate quotient), and atan(u) = u + u^3 P(u^2) with an 11-term Chebyshev fit on
// [0, tan^2(pi/8)] (approximation error 2^-57, f64 evaluation ~2^-53; tools/atan2_coefs.py).  Its
// relative error is below 2^-50, so RN_f32(A) equals RN_f32 of any f64 atan2 within an ulp of the
// true angle unless A lies within 128 f64 ulps of an f32 rounding midpoint: `near` flags those
// (and zeros, tiny and non-finite cases) for the caller's fallback to the library call.
constexpr double ATAN_P[11] = {-0x1.3a31b1c0fd3b7p-6, 0x1.4162c02b1dda3p-5, -0x1.a0999c632b6edp-5,
                               0x1.dfe6497e96323p-5, -0x1.10fa77b1a6d57p-4, 0x1.3b1263064f6b9p-4,
                               -0x1.745d0b28a7e37p-4, 0x1.c71c71853d7fap-4, -0x1.2492492436201p-3,
                               0x1.999999999934cp-3, -0x1.5555555555555p-2};
constexpr double PI_F64 = 0x1.921fb54442d18p+1, PI_2_F64 = 0x1.921fb54442d18p+0, PI_4_F64 = 0x1.921fb54442d18p-1;
constexpr double TAN_PI_8 = 0x1.a827999fcef32p-2;

struct Atan2 { float f; bool near; };
__device__ __forceinline__ Atan2 atan2_core(float yf, float xf) {
    const double x = (double)xf, y = (double)yf;
    const double ax = fabs(x), ay = fabs(y);
    const double mx = fmax(ax, ay), mn = fmin(ax, ay);
    const bool big = mn > TAN_PI_8 * mx;
    const double num = big ? mn - mx : mn, den = big ? mn + mx : mx;
    double r = __builtin_amdgcn_rcp(den);
    r = __builtin_fma(__builtin_fma(-den, r, 1.0), r, r);
    r = __builtin_fma(__builtin_fma(-den, r, 1.0), r, r);
    double u = num * r;
    u = __builtin_fma(__builtin_fma(-den, u, num), r, u);
    const double s = u * u;
    // Horner with each coefficient an SGPR-pair operand of v_fma_f64 (two s_mov_b32 on the scalar unit):
    // the compiler's own form, v_fmac_f64 with the coefficient first moved into the accumulator's VGPR
    // pair, issues 20 more VALU instructions per wave
    double p = ATAN_P[0];
#pragma unroll
    for (int k = 1; k < 11; ++k) {
        double q;
        asm("v_fma_f64 %0, %1, %2, %3" : "=v"(q) : "v"(p), "v"(s), "s"(ATAN_P[k]));
        p = q;
    }
    double a = __builtin_fma(u * s, p, u);
    a = big ? a + PI_4_F64 : a;
    a = ay > ax ? PI_2_F64 - a : a;
    a = __builtin_signbit(x) ? PI_F64 - a : a;
    a = __builtin_copysign(a, y);
    const float f = (float)a;
    // Distance of A to the nearest f32 rounding midpoint, in f64 ulps of A: for a normal f32 result the
    // conversion keeps A's top 24 significand bits and rounds on the low 29, so every midpoint of A's
    // binade -- including the one below a power of two the result may round up to -- sits at low29 =
    // 2^28.  Flag |low29 - 2^28| <= 128 ulps (>= 2^-46 |A|; the core's error is below 2^-50 |A|, 8 ulps,
    // the library's below an ulp): one integer compare instead of the f64 distance arithmetic (frexp,
    // ldexp, three f64 subtractions).
    const uint32_t lo = (uint32_t)__builtin_bit_cast(uint64_t, a) & 0x1FFFFFFFu;
    const bool mid = lo - (0x10000000u - 128u) <= 256u;
    const bool near = (x != x) || (y != y) || !(mx > 0.0 && mx < 0x1p200) || !(fabs(a) >= 0x1p-120) || mid;
    return {f, near};
}

}  // namespace crm
}  // namespace bh
