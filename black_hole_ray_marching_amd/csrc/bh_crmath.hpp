// bh_crmath.hpp — correctly rounded f32 division and square root for gfx950, cheap forms.
//
// hipcc's IEEE division expands to 11 VALU ops (v_div_scale x2, v_rcp, 6 FMA-class ops, v_div_fmas,
// v_div_fixup) and measures ~50 cycles per wave-instruction stream on MI355X; its IEEE sqrt ~54
// (tools/ubench/valu_rates.hip).  The march loop needs 18 divisions and 7 square roots per RK step,
// so these dominate the exact (bit-parity) kernel.  The forms below drop the scaling/fix-up steps,
// which only act on operands near the ends of the exponent range, and share one refined reciprocal
// between the three divisions of rd_derivative.  Each form is the SAME arithmetic as hipcc's
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
// v_sqrt_f32 is within 1 ulp for inputs >= 2^-96; one residual test on each neighbour picks the
// correctly rounded value (LLVM's lowering of an IEEE fsqrt without its small-input scaling).
// Exact for x >= 2^-96 (incl. +inf), x == +-0, and NaN/negative -> NaN.
constexpr float SQRT_MIN = 0x1p-96f;

__device__ __forceinline__ float sqrt_core(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    float r = (rm <= 0.0f) ? sm : s;
    r = (rp > 0.0f) ? sp : r;
    return r;
}
// unsafe iff 0 <= x < 2^-96 (x == 0 is exact too, but rare; it just takes the IEEE path)
__device__ __forceinline__ bool sqrt_bad(float x) { return x < SQRT_MIN; }

// ---- division by a shared denominator ---------------------------------------------------------
// Markstein sequence of hipcc's IEEE division with the div_scale / div_fmas scaling left out:
//   r0 = rcp(d); r = r0 + r0*(1 - d*r0); y = n*r; y += r*(n - d*y); q = y + r*(n - d*y)
// Correctly rounded when d and n/d are normal and far from the exponent limits and |n| is not tiny
// (the residual n - d*y must not underflow).  The caller guarantees:
//   DIV_D_MIN <= d <= DIV_D_MAX  (checked per denominator, div_d_bad)
//   n == 0 or DIV_N_MIN <= |n| <= 2^64
// The residuals are formed negated, e' = d*y - n = -(n - d*y) (exact in an FMA, RN is symmetric),
// and added back as fma(-e', r, y): identical for n != 0, and for n = +-0 every sum then keeps the
// IEEE sign of the zero quotient (-0 + -0 = -0) without a copysign.
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
__device__ __forceinline__ float div_core(float n, const Rcp& R) {
    const float y = n * R.r;
    const float e1 = __builtin_fmaf(R.d, y, -n);
    const float y1 = __builtin_fmaf(-e1, R.r, y);
    const float e2 = __builtin_fmaf(R.d, y1, -n);
    return __builtin_fmaf(-e2, R.r, y1);
}
__device__ __forceinline__ bool div_d_bad(float d) { return !(d >= DIV_D_MIN && d <= DIV_D_MAX); }

// ---- division by 6 ----------------------------------------------------------------------------
// y = x * RN(1/6); q = y + RN(1/6) * (x - 6y): equals RN(x / 6) for every x whose quotient is not
// subnormal (exhaustively checked over all 2^32 inputs; the residual is formed negated as in
// div_core so that x = +-0 gives the IEEE zero).  Callers guarantee x == 0 or |x| >= DIV_N_MIN.
__device__ __forceinline__ float div6(float x) {
    constexpr float R6 = 1.0f / 6.0f;
    const float y = x * R6;
    const float e = __builtin_fmaf(y, 6.0f, -x);
    return __builtin_fmaf(-e, R6, y);
}

// ---- numerator magnitude guard ----------------------------------------------------------------
// x / 12 = (x / 6) / 2: halving is exact for the normal quotients of the div6 domain, so this is
// RN(x / 12) wherever div6 is RN(x / 6) (checked exhaustively as selftest op 5).
__device__ __forceinline__ float div12(float x) { return div6(x) * 0.5f; }

// key(n) = 2*bits(|n|) - 1 (mod 2^32): +-0 -> 0xFFFFFFFF, tiny -> small, so key(n) < KEY_MIN iff
// 0 < |n| < DIV_N_MIN; a running v_min3_u32 over keys needs one compare per step.  (A float
// min of |n| would be one op cheaper but cannot tell 0 from tiny: measured 2x slower overall,
// because every camera-A ray starts on two coordinate planes and its first step then re-runs.)
constexpr uint32_t KEY_MIN = (0x21800000u << 1) - 1u;  // key(2^-60)
__device__ __forceinline__ uint32_t key(float n) { return (__float_as_uint(n) << 1) - 1u; }
__device__ __forceinline__ uint32_t kmin3(uint32_t a, uint32_t b, uint32_t c) { return min(min(a, b), c); }

}  // namespace crm
}  // namespace bh
