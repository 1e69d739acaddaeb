// bh_srgb.hpp — linear f32 -> sRGB byte, the store of a Bgra8UnormSrgb render target (the reference's
// surface/consumer format: src/scene.rs:259-274, src/copy.rs:132, src/remix.rs:160).
//
// Normative encode (oracle/bh_oracle.c bho_srgb_encode): clamp to [0, 1] (NaN -> 0), the sRGB OETF in
// double, round half up to 0..255.  It is monotone in x, so it is fully described by 255 thresholds:
// T[k] = the smallest float with code >= k (bh_host.cpp builds them from the definition; T[0] = 0,
// T[256] = +inf).  On the GPU a hardware-log2/exp2 evaluation of the OETF lands within one code of
// the answer, and the two neighbouring thresholds fix it: exact for every float (checked
// exhaustively on the device, bh_selftest_crmath op 4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bh {

constexpr int SRGB_TABLE = 257;

__device__ __forceinline__ uint32_t srgb_encode(float x, const float* T) {
    const float xc = fminf(fmaxf(x, 0.0f), 1.0f);  // fmaxf(NaN, 0) = 0
    const float s = xc <= 0.0031308f ? 12.92f * xc
                                     : 1.055f * __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(xc) * (1.0f / 2.4f)) - 0.055f;
    int c = (int)(s * 255.0f + 0.5f);
    c = c < 0 ? 0 : (c > 255 ? 255 : c);
    c = (xc < T[c]) ? c - 1 : c;        // T[0] = 0 <= xc: never below 0
    c = (xc >= T[c + 1]) ? c + 1 : c;   // T[256] = +inf: never above 255
    return (uint32_t)c;
}

// Table form without log2/exp2 (the bloom chain stores ~9 channels per pixel): on [2^-13, 1) every
// bucket of 2^-7 relative width (7 mantissa bits) spans at most one code boundary, so the code is
// the bucket's base code B[i] (the code of its lower end) plus one where x reaches T[B[i] + 1].
// Below 2^-13 the code is 0 (T[1] > 2^-13), which bucket 0 already gives.  Exhaustively checked on
// the device (bh_selftest_crmath op 6).  The host builds B from T (bh_host.cpp).
constexpr uint32_t SRGB_BUCKET_SHIFT = 16;
constexpr uint32_t SRGB_BUCKET_BASE = (127u - 13u) << 7;  // bucket index of 2^-13
constexpr int SRGB_BUCKETS = 13 * 128;                   // [2^-13, 1)

__device__ __forceinline__ uint32_t srgb_encode_lut(float x, const uint8_t* B, const float* T) {
    const float xc = fminf(fmaxf(x, 0.0f), 1.0f);  // fmaxf(NaN, 0) = 0
    int32_t i = (int32_t)(__float_as_uint(xc) >> SRGB_BUCKET_SHIFT) - (int32_t)SRGB_BUCKET_BASE;
    i = i < 0 ? 0 : (i > SRGB_BUCKETS - 1 ? SRGB_BUCKETS - 1 : i);
    const uint32_t c = B[i];
    return c + (xc >= T[c + 1] ? 1u : 0u);
}

// Code-table form (one LDS read instead of two dependent ones): within a bucket every float shares its
// upper 16 bits, so the one threshold a bucket may hold is fixed by its low 16 bits.  Entry i =
// base code | thr17 << 15, thr17 = the threshold's low 16 bits, or 0x10000 (never reached) when the
// bucket holds none: code = base + (low16(x) >= thr17).  Entry SRGB_BUCKETS is 1.0 (code 255); values
// below 2^-13 clamp to entry 0, which holds no threshold (T[1] > 2^-13 * (1 + 2^-7)).  Built by the host
// (bh_host.cpp, bh_srgb_code_table); exhaustively checked on the device (bh_selftest_crmath op 10).
constexpr int SRGB_CODES = SRGB_BUCKETS + 1;
__device__ __forceinline__ uint32_t srgb_encode_code(float x, const uint32_t* E) {
    const float xc = fminf(fmaxf(x, 0.0f), 1.0f);  // fmaxf(NaN, 0) = 0
    const uint32_t b = __float_as_uint(xc);
    int32_t i = (int32_t)(b >> SRGB_BUCKET_SHIFT) - (int32_t)SRGB_BUCKET_BASE;
    i = i < 0 ? 0 : (i > SRGB_BUCKETS ? SRGB_BUCKETS : i);
    const uint32_t e = E[i];
    return (e & 0xFFu) + ((b & 0xFFFFu) >= (e >> 15) ? 1u : 0u);
}

// BGRA8 texel (byte 0 = B) of linear rgb, alpha 1.
__device__ __forceinline__ uint32_t srgb_bgra8(float r, float g, float b, const float* T) {
    return srgb_encode(b, T) | (srgb_encode(g, T) << 8) | (srgb_encode(r, T) << 16) | 0xFF000000u;
}

}  // namespace bh
