// bh_bloom.hip — the reference's post-processing chain (Kawase bloom + remix)
// on BGRA8-sRGB images: the consumer of the march kernel's two targets (bh_render with
// BH_OUT_BGRA8_SRGB), replacing Bloom::render (src/bloom.rs:53-71).
//
// Semantics: oracle/bh_bloom_oracle.c is the pass-by-pass restatement (every texture Bgra8UnormSrgb:
// each pass decodes its inputs through the sRGB table, filters in f32, and stores through the exact
// encoder of bh_srgb.hpp).  Two schedules produce the same bytes:
//   * literal: one kernel per render pass of the reference, in its order, into the same textures;
//   * fused (default when it is exact): a same-size pass samples its input exactly at texel centres
//     when u = RN((x+0.5)/w) gives RN(u*w) - 0.5 == x for every x (and likewise y) -- then a copy is
//     the identity and a 1:1 remix input can be read at the pixel itself.  The host checks that
//     for every size involved (true for power-of-two frames such as 4096x2048); the chain then
//     collapses to 6 kernels: Y = X + 0.5 blur1(X) (one pass, computed once: the reference's
//     second loop iteration recomputes the same Y from the same input), two 2:1 downsamples, two
//     upsamples at 1/2 and full size, and out = col + 0.5 (Y + 0.5 up(U0)) (one pass).  Each fused
//     stage still quantises through the sRGB encode exactly where the reference stores a texture.
// Byte work bound by the exact filter arithmetic and its LDS reads, not by HBM: one lane per output
// pixel (a 2x2 quad in the 2:1 up passes), each block's input footprint decoded into LDS once,
// coalesced stores; the 256-entry decode table and the 257 encode thresholds in LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>
#include <utility>

#include "bh_common.hpp"
#include "bh_crmath.hpp"
#include "bh_srgb.hpp"

namespace bh {
namespace bloom {

struct Tex {
    uint32_t* px;  // BGRA8 texels, row-major, tightly packed
    uint32_t w, h;
};
struct CTex {
    const uint32_t* px;
    uint32_t w, h;
};

struct F4 { float r, g, b, a; };

// Block coordinates with the 8 XCDs' L2s in mind.  The dispatcher hands linear workgroup b to XCD
// b % 8, so in the raw grid neighbouring blocks -- which stage overlapping halo footprints of the same
// texture -- run on different XCDs, and every XCD fetches its blocks' footprints through its own L2.
// Remapped, XCD k processes the k-th eighth of the grid in row-major order (the remainder, fewer than
// 8 blocks, keeps the raw order): adjacent blocks share an L2.  A bijection of the grid; results never
// depend on it.
__device__ __forceinline__ uint2 xcd_block() {
    const uint32_t gx = gridDim.x, n = gx * gridDim.y;
    const uint32_t b = blockIdx.y * gx + blockIdx.x, per = n >> 3;
    const uint32_t t = b < (per << 3) ? (b & 7u) * per + (b >> 3) : b;
    const uint32_t ty = t / gx;
    return make_uint2(t - ty * gx, ty);
}

// LDS tables of a block: sRGB decode (256), alpha decode k/255 (256) and the encoder: its thresholds
// (257) and base codes (table form, bh_srgb.hpp).  (Measured and not kept, DESIGN.md §7b: the encoder's
// code table -- one read per channel instead of two dependent ones -- and the alpha decode from constant
// memory instead of LDS.)
struct Lds {
    float lut[256];
    float alut[256];
    float T[SRGB_TABLE];
    uint32_t B32[SRGB_BUCKETS / 4];
};
struct Tables {
    const float* lut;      // 256
    const float* enc;      // 257
    const uint8_t* bkt;    // SRGB_BUCKETS
    const uint32_t* code;  // SRGB_CODES
};
__device__ __forceinline__ void load_tables(Tables tb, Lds& L) {
    L.lut[threadIdx.x] = tb.lut[threadIdx.x];
    L.alut[threadIdx.x] = (float)threadIdx.x / 255.0f;
    L.T[threadIdx.x] = tb.enc[threadIdx.x];
    if (threadIdx.x == 0) L.T[256] = tb.enc[256];
    const uint32_t* b = reinterpret_cast<const uint32_t*>(tb.bkt);
    for (uint32_t i = threadIdx.x; i < SRGB_BUCKETS / 4; i += 256) L.B32[i] = b[i];
    __syncthreads();
}

// A1: the caller knows the texel's alpha byte is 255 (a block whose inputs are all opaque, see
// with_source): alpha decodes to 1.0 without a table read, and the compiler folds the alpha channel's
// whole arithmetic (sums, x/12, the encoder) to constants
// Block-wide AND of a predicate at a barrier the caller needs anyway: one ballot per wave, its lane 0's
// word in LDS, the barrier, then every thread reads the 4 words (__syncthreads_and costs an LDS atomic
// per thread on one address).
__device__ __forceinline__ bool barrier_and(bool p) {
    __shared__ uint32_t w[4];
    const bool all = __builtin_amdgcn_ballot_w64(!p) == 0ull;
    if ((threadIdx.x & 63u) == 0u) w[threadIdx.x >> 6] = all ? 1u : 0u;
    __syncthreads();
    return (w[0] & w[1] & w[2] & w[3]) != 0u;
}
template <bool A1 = false>
__device__ __forceinline__ F4 dec(const Lds& L, uint32_t t) {
    return {L.lut[(t >> 16) & 0xffu], L.lut[(t >> 8) & 0xffu], L.lut[t & 0xffu], A1 ? 1.0f : L.alut[t >> 24]};
}
// lo <= hi: one v_med3_i32
__device__ __forceinline__ int32_t clampi(int32_t v, int32_t lo, int32_t hi) { return min(max(v, lo), hi); }

__device__ __forceinline__ uint32_t unorm8(float a) {
    // branch-free: the conversion of an out-of-range a is discarded by the selects
    const uint32_t v = (uint32_t)__double2int_rd((double)fminf(fmaxf(a, 0.0f), 1.0f) * 255.0 + 0.5);
    return !(a > 0.0f) ? 0u : (a >= 1.0f ? 255u : v);
}
// the Bgra8UnormSrgb store of a pass's result
__device__ __forceinline__ uint32_t enc(const Lds& L, F4 c) {
    const uint8_t* B = reinterpret_cast<const uint8_t*>(L.B32);
    return srgb_encode_lut(c.b, B, L.T) | (srgb_encode_lut(c.g, B, L.T) << 8) | (srgb_encode_lut(c.r, B, L.T) << 16) |
           (unorm8(c.a) << 24);
}
template <bool A1 = false>
__device__ __forceinline__ F4 quant(const Lds& L, F4 c) { return dec<A1>(L, enc(L, c)); }

// Texcoord of pixel i of an n-pixel axis, (i + 0.5) / n: the correctly rounded division core with the
// reciprocal of n shared by the block (exact: n >= 1 and i + 0.5 >= 0.5 are inside its domain).
__device__ __forceinline__ float texcoord(uint32_t i, const crm::Rcp& R) { return crm::div_core((float)i + 0.5f, R); }

// x / 12 of the up-sampling filter, for the four channels of a sum: the div12 core where it is exact
// (x == 0 or |x| >= 2^-60, selftest op 5), IEEE division for all four when any channel of any lane is
// outside that (never taken by sums of decoded texels).  One test after all four cores keeps the sums'
// arithmetic in one basic block: a branch per channel let the compiler sink the other channels' sums
// past it, keeping every tap's texels live.
__device__ __forceinline__ F4 div12(const F4& s) {
    F4 q{crm::div12(s.r), crm::div12(s.g), crm::div12(s.b), crm::div12(s.a)};
    const uint32_t k = crm::kmin3(crm::key(s.r), crm::key(s.g), min(crm::key(s.b), crm::key(s.a)));
    if (__builtin_expect(k < crm::KEY_MIN, 0)) q = {s.r / 12.0f, s.g / 12.0f, s.b / 12.0f, s.a / 12.0f};
    return q;
}

// Texel sources: decoded texel (x, y) of a BGRA8 texture straight from global memory, or from a
// block's LDS tile of pre-decoded texels covering exactly the footprint the block samples.
struct GlobalSrc {
    static constexpr bool kA1 = false;
    CTex t;
    const Lds* L;
    __device__ __forceinline__ F4 at(int32_t x, int32_t y) const { return dec(*L, t.px[(uint32_t)y * t.w + x]); }
};
template <int FP>
struct TileSrc {
    static constexpr bool kA1 = false;
    CTex t;
    const float4* tile;  // decoded texels [y0, y0 + FP) x [x0, x0 + FP)
    int32_t x0, y0;
    __device__ __forceinline__ F4 at(int32_t x, int32_t y) const {
        const float4 v = tile[(y - y0) * FP + (x - x0)];
        return {v.x, v.y, v.z, v.w};
    }
};

// clamp-to-edge bilinear of decoded texels at texcoord (u, v) (oracle: sample)
// (t is never NaN: texcoords come from pixel indices) fminf(fmaxf(t, -1), n) as one v_med3_f32
__device__ __forceinline__ float sample_coord(float u, uint32_t n) {
    const float t = u * (float)n - 0.5f;
    return __builtin_amdgcn_fmed3f(t, -1.0f, (float)n);
}
template <class Src>
__device__ __forceinline__ F4 sample(const Src& src, float u, float v) {
    const CTex t = src.t;
    const float tx = sample_coord(u, t.w), ty = sample_coord(v, t.h);
    const float fx0 = floorf(tx), fy0 = floorf(ty);
    const float fa = tx - fx0, fb = ty - fy0;
    const int32_t wm = (int32_t)t.w - 1, hm = (int32_t)t.h - 1;
    int32_t x0 = (int32_t)fx0, y0 = (int32_t)fy0;
    const int32_t x1 = clampi(x0 + 1, 0, wm), y1 = clampi(y0 + 1, 0, hm);
    x0 = clampi(x0, 0, wm);
    y0 = clampi(y0, 0, hm);
    const F4 t00 = src.at(x0, y0), t10 = src.at(x1, y0), t01 = src.at(x0, y1), t11 = src.at(x1, y1);
    const float ia = 1.0f - fa, ib = 1.0f - fb;
    F4 r;
    r.r = (t00.r * ia + t10.r * fa) * ib + (t01.r * ia + t11.r * fa) * fb;
    r.g = (t00.g * ia + t10.g * fa) * ib + (t01.g * ia + t11.g * fa) * fb;
    r.b = (t00.b * ia + t10.b * fa) * ib + (t01.b * ia + t11.b * fa) * fb;
    r.a = (t00.a * ia + t10.a * fa) * ib + (t01.a * ia + t11.a * fa) * fb;
    return r;
}

// The same sample when its bilinear weights are exactly 0 (tx and ty integral or clamped): the lerps
// then return texel (x0, y0) bit for bit (t * 1 + t' * 0 == t for finite t >= 0).  The host proves
// this per tap for every pixel of a launch (bloom_point_mask) before a kernel may take it.
template <class Src>
__device__ __forceinline__ F4 sample_point(const Src& src, float u, float v) {
    const CTex t = src.t;
    const int32_t x0 = clampi((int32_t)floorf(sample_coord(u, t.w)), 0, (int32_t)t.w - 1);
    const int32_t y0 = clampi((int32_t)floorf(sample_coord(v, t.h)), 0, (int32_t)t.h - 1);
    return src.at(x0, y0);
}

// kawase_upsample.wgsl:25-38: 8 taps around uv at offsets (mx, my) * 0.5/res * 3 for
// (mx, my) = (-2,0), (-1,1), (0,2), (1,1), (2,0), (1,-1), (0,-2), (-1,-1), weights 1,2,1,2,.., / 12.
// (hx * m) * 3 is exactly the shader's (-hx * 2.0) * 3, (-hx) * 3, 0.0 * 3, ... (negation and doubling
// are exact), so the taps can be generated in a rolled loop: 8 unrolled taps keep 160 VGPRs live.
struct Taps {
    float hx, hy;
    __device__ __forceinline__ Taps(uint32_t rx, uint32_t ry) : hx(0.5f / (float)rx), hy(0.5f / (float)ry) {}
    __device__ __forceinline__ float du(int i) const { return (hx * (float)((int)((0x12343210u >> (4 * i)) & 15u) - 2)) * 3.0f; }
    __device__ __forceinline__ float dv(int i) const { return (hy * (float)((int)((0x10123432u >> (4 * i)) & 15u) - 2)) * 3.0f; }
    // extreme offsets (taps 0 / 4 along u, 6 / 2 along v)
    __device__ __forceinline__ float du_min() const { return du(0); }
    __device__ __forceinline__ float du_max() const { return du(4); }
    __device__ __forceinline__ float dv_min() const { return dv(6); }
    __device__ __forceinline__ float dv_max() const { return dv(2); }
};
// tap i's offset multiplier along an axis (Taps::du / dv), and floor / remainder in eighths (the
// standard plans, see quad_tap_std)
__host__ __device__ constexpr int tap_m(int axis, int i) {
    return (int)(((axis ? 0x10123432u : 0x12343210u) >> (4 * i)) & 15u) - 2;
}
__host__ __device__ constexpr int fdiv8(int v) { return v >= 0 ? v / 8 : -((7 - v) / 8); }
__host__ __device__ constexpr int fmod8(int v) { return v - 8 * fdiv8(v); }

// The structured form of an 8-tap pass, proven by the host for every pixel of a launch
// (bh_bloom_tap_plan): along each axis tap i's unclamped texel coordinate u*n - 0.5 equals x + o_i + f_i
// exactly, with an integer offset o_i and a weight f_i of 0 (point) or 1/2 (half).  The bilinear sample
// then reads texels clamp(x + o_i) and clamp(x + o_i + 1) at constant offsets, and its lerps reduce
// exactly: with weights 1/2 (products by 1/2 exact for the decoded texels, which are 0 or >= 2^-12)
//   (t0 * 0.5 + t1 * 0.5) == (t0 + t1) * 0.5,   both axes: ((t00 + t10) + (t01 + t11)) * 0.25,
// and with weight 0 the lerp returns t0 (t * 1 + t' * 0 == t).  Clamping agrees at the edges: a
// coordinate clamped to -1 or n has weight 0 and selects the edge texel, which both reads of a half
// tap then clamp to (t + t) * 0.5 == t).
struct TapPlan {
    int32_t ox[8], oy[8];
    uint32_t hx, hy;                 // bit i: tap i's weight along x (y) is 1/2, else 0
    int32_t lo_x, hi_x, lo_y, hi_y;  // the footprint's offsets: min o_i, max (o_i + half_i)
    uint32_t valid;
};
// A block's staged footprint for a TapPlan: entry (y - y0) * FP + (x - x0) of the tile holds texel
// (clamp(x), clamp(y)) for the logical coordinates [x0, x0 + FP) x [y0, y0 + FP): decoded (float4), or
// with RAW the BGRA8 word (4 B instead of 16: the final pass's 44 x 44 footprint then takes 7.6 KiB of
// LDS instead of 30 KiB, so twice as many blocks fit a CU), decoded when a tap reads it.
template <int FP, bool RAW = false, int STD = 0, bool A1 = false>
struct PlanSrc {
    static constexpr bool kA1 = A1;
    CTex t;
    const void* tile;
    int32_t x0, y0;
    const TapPlan* P;
    const Lds* L;
    int32_t px, py;  // the pixel this thread computes (up8)
    __device__ __forceinline__ float4 fetch(int32_t i) const {
        if constexpr (RAW) {
            const F4 d = dec<A1>(*L, static_cast<const uint32_t*>(tile)[i]);
            return make_float4(d.r, d.g, d.b, d.a);
        } else {
            const float4 v = static_cast<const float4*>(tile)[i];
            return make_float4(v.x, v.y, v.z, A1 ? 1.0f : v.w);
        }
    }
    __device__ __forceinline__ F4 at(int32_t x, int32_t y) const {
        const float4 v = fetch((y - y0) * FP + (x - x0));
        return {v.x, v.y, v.z, v.w};
    }
};

// up8's sums, tap by tap: s + q * w with w = 1 (even taps) or 2 (odd taps).  q * 2 is exact for every
// finite q, so RN(s + RN(q * 2)) == fma(q, 2, s): one instruction per channel instead of two.
__device__ __forceinline__ void acc(F4& s, const F4& q, int i) {
    if (i == 0) {
        s = q;
    } else if (i & 1) {
        s.r = __builtin_fmaf(q.r, 2.0f, s.r); s.g = __builtin_fmaf(q.g, 2.0f, s.g);
        s.b = __builtin_fmaf(q.b, 2.0f, s.b); s.a = __builtin_fmaf(q.a, 2.0f, s.a);
    } else {
        s.r = s.r + q.r; s.g = s.g + q.g; s.b = s.b + q.b; s.a = s.a + q.a;
    }
}
// A TapPlan tap's contribution, exactly: the half-weight forms reduce a tap to h * 2^-k with h a sum of
// decoded texels (0 or >= 2^-12, so every product by a power of two below is exact), and the tap's
// weight w = 1 or 2 then folds into one fma:  s + RN(h * 0.5) * 2 == s + h,  s + RN(h * 0.5) ==
// fma(h, 0.5, s),  s + RN(h * 0.25) * 2 == fma(h, 0.5, s),  s + RN(h * 0.25) == fma(h, 0.25, s).
// `sh` = the tap's scale exponent k (0: a point tap, 1: one half axis, 2: both).
__device__ __forceinline__ void acc_scaled(F4& s, const float4& h, int sh, int i) {
    const float sc = sh == 0 ? 1.0f : (sh == 1 ? 0.5f : 0.25f);
    if (i == 0) {
        s = {h.x * sc, h.y * sc, h.z * sc, h.w * sc};
        return;
    }
    const int e = sh - (i & 1);  // s gains h * 2^-e, exactly
    if (e == 0) {
        s.r = s.r + h.x; s.g = s.g + h.y; s.b = s.b + h.z; s.a = s.a + h.w;
    } else {
        const float m = e < 0 ? 2.0f : (e == 1 ? 0.5f : 0.25f);
        s.r = __builtin_fmaf(h.x, m, s.r); s.g = __builtin_fmaf(h.y, m, s.g);
        s.b = __builtin_fmaf(h.z, m, s.b); s.a = __builtin_fmaf(h.w, m, s.a);
    }
}

// `point`: bit i set = tap i's weights are exactly 0 for every pixel of this launch
template <class Src>
__device__ __forceinline__ F4 up8(const Src& src, const Taps& k, float u, float v, uint32_t point) {
    F4 s = (point & 1u) ? sample_point(src, u + k.du(0), v + k.dv(0)) : sample(src, u + k.du(0), v + k.dv(0));
#pragma unroll
    for (int i = 1; i < 8; i++) {
        // the sched barrier keeps one tap in flight at a time: all 8 unrolled taps hoisted together
        // take 160 VGPRs (3 waves per SIMD); the rolled loop recomputes the offsets every tap
        __builtin_amdgcn_sched_barrier(0);
        const float tu = u + k.du(i), tv = v + k.dv(i);
        acc(s, ((point >> i) & 1u) ? sample_point(src, tu, tv) : sample(src, tu, tv), i);
    }
    return div12(s);
}
// up8 over a TapPlan-staged footprint: the same sums, each tap 1, 2 or 4 LDS reads at constant offsets
// (STD: the standard plan A = STD, its offsets and halves constants -- see quad_tap_std)
template <int FP, bool RAW, int STD, bool A1>
__device__ __forceinline__ F4 up8(const PlanSrc<FP, RAW, STD, A1>& src, const Taps&, float, float, uint32_t) {
    const TapPlan& P = *src.P;
    const int32_t base = (src.py - src.y0) * FP + (src.px - src.x0);
    F4 s{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int32_t o = base + (STD ? fdiv8(STD * tap_m(1, i)) * FP + fdiv8(STD * tap_m(0, i)) : P.oy[i] * FP + P.ox[i]);
        float4 q = src.fetch(o);
        const bool hx = STD ? fmod8(STD * tap_m(0, i)) == 4 : (P.hx >> i) & 1u;
        const bool hy = STD ? fmod8(STD * tap_m(1, i)) == 4 : (P.hy >> i) & 1u;
        if (hx && hy) {
            const float4 a = src.fetch(o + 1), b = src.fetch(o + FP), c = src.fetch(o + FP + 1);
            q = make_float4((q.x + a.x) + (b.x + c.x), (q.y + a.y) + (b.y + c.y), (q.z + a.z) + (b.z + c.z),
                            (q.w + a.w) + (b.w + c.w));
            acc_scaled(s, q, 2, i);
        } else if (hx || hy) {
            const float4 a = src.fetch(o + (hx ? 1 : FP));
            acc_scaled(s, make_float4(q.x + a.x, q.y + a.y, q.z + a.z, q.w + a.w), 1, i);
        } else {
            acc_scaled(s, q, 0, i);
        }
    }
    return div12(s);
}

// the 16 sums complete here (an empty asm that reads them): keeps the compiler from sinking part of a
// tap's arithmetic below later taps, which would keep every tap's texels live at once (~240 VGPRs)
__device__ __forceinline__ void pin(F4 (&s)[2][2]) {
    asm volatile("" ::"v"(s[0][0].r), "v"(s[0][0].g), "v"(s[0][0].b), "v"(s[0][0].a), "v"(s[0][1].r), "v"(s[0][1].g),
                 "v"(s[0][1].b), "v"(s[0][1].a), "v"(s[1][0].r), "v"(s[1][0].g), "v"(s[1][0].b), "v"(s[1][0].a),
                 "v"(s[1][1].r), "v"(s[1][1].g), "v"(s[1][1].b), "v"(s[1][1].a));
}
// remix.wgsl:22-24
// c1 * 0.5 is exact (c1 a sum / lerp of decoded texels: 0 or far above the subnormals), so
// c0 + RN(c1 * 0.5) == fma(c1, 0.5, c0)
__device__ __forceinline__ F4 remix(F4 c0, F4 c1) {
    return {__builtin_fmaf(c1.r, 0.5f, c0.r), __builtin_fmaf(c1.g, 0.5f, c0.g), __builtin_fmaf(c1.b, 0.5f, c0.b),
            __builtin_fmaf(c1.a, 0.5f, c0.a)};
}

enum Shader : uint32_t { SH_COPY = bh_bloom_shader_copy, SH_DOWN = bh_bloom_shader_down, SH_UP = bh_bloom_shader_up,
                         SH_REMIX = bh_bloom_shader_remix };

// The texel range one axis of a 16-pixel block samples through 8 taps: every rounding step of
// sample_coord is monotone in the texcoord, so the extreme taps of the first and last pixel bound it.
struct Span { int32_t lo, n; };
__device__ __forceinline__ Span tap_span(uint32_t first, uint32_t last, const crm::Rcp& R, float dmin, float dmax,
                                         uint32_t tn) {
    const float a = sample_coord(texcoord(first, R) + dmin, tn), b = sample_coord(texcoord(last, R) + dmax, tn);
    const int32_t hi_lim = (int32_t)tn - 1;
    const int32_t lo = clampi((int32_t)floorf(a), 0, hi_lim), hi = clampi((int32_t)floorf(b) + 1, 0, hi_lim);
    return {lo, hi - lo + 1};
}

// Run `body(src)` with the block's input footprint staged in LDS (decoded) when it fits FP x FP,
// else straight from global memory; both give identical values.  Called by every thread.  RAW: a
// TapPlan footprint is staged as BGRA8 words (PlanSrc<FP, true>; `tile` then needs FP*FP*4 bytes,
// else FP*FP*16).  It also loads the block's tables (load_tables), after issuing the footprint's loads:
// the two global round trips overlap instead of following each other.  In the TapPlan form a block
// whose staged texels (and the caller's `opaque` inputs of every thread) all have alpha byte 255 runs
// `body` with an A1 source (PlanSrc<..., true>: see dec): alpha is then 1.0 everywhere and its arithmetic
// folds away.  Both forms give the same bytes.
template <int FP, bool RAW = false, int STD = 0, class Body>
__device__ __forceinline__ void with_source(Tables tb, CTex t, Lds& L, float4* tile, const Taps& k, uint32_t ow,
                                            uint32_t oh, const crm::Rcp& Rw, const crm::Rcp& Rh, const TapPlan& P,
                                            Body body, bool opaque = false) {
    const uint32_t bx = xcd_block().x * 16u, by = xcd_block().y * 16u;
    if (P.valid && P.hi_x - P.lo_x + 16 <= FP && P.hi_y - P.lo_y + 16 <= FP) {  // launch-uniform
        // the footprint with clamp-to-edge addressing: row r of the tile is texel row clamp(y0 + r);
        // every load of this thread first, then the decodes
        const int32_t x0 = (int32_t)bx + P.lo_x, y0 = (int32_t)by + P.lo_y;
        const int32_t nx = P.hi_x - P.lo_x + 16, ny = P.hi_y - P.lo_y + 16;
        const int32_t tx = (int32_t)(threadIdx.x & 15u), ty = (int32_t)(threadIdx.x >> 4);
        constexpr int R = (FP + 15) / 16;
        const int32_t wm = (int32_t)t.w - 1, hm = (int32_t)t.h - 1;
        uint32_t raw[R][R];
#pragma unroll
        for (int a = 0; a < R; ++a)
#pragma unroll
            for (int b = 0; b < R; ++b) {
                const int32_t ly = ty + 16 * a, lx = tx + 16 * b;
                raw[a][b] = 0xFF000000u;
                if (ly < ny && lx < nx)
                    raw[a][b] = t.px[(uint32_t)clampi(y0 + ly, 0, hm) * t.w + clampi(x0 + lx, 0, wm)];
            }
        load_tables(tb, L);
#pragma unroll
        for (int a = 0; a < R; ++a)
#pragma unroll
            for (int b = 0; b < R; ++b) {
                const int32_t ly = ty + 16 * a, lx = tx + 16 * b;
                if (ly < ny && lx < nx) {
                    if constexpr (RAW) {
                        reinterpret_cast<uint32_t*>(tile)[ly * FP + lx] = raw[a][b];
                    } else {
                        const F4 d = dec(L, raw[a][b]);
                        tile[ly * FP + lx] = make_float4(d.r, d.g, d.b, d.a);
                    }
                }
            }
        uint32_t m = 0xFFFFFFFFu;
#pragma unroll
        for (int a = 0; a < R; ++a)
#pragma unroll
            for (int b = 0; b < R; ++b) m = min(m, raw[a][b]);
        const bool a1 = barrier_and(opaque && m >= 0xFF000000u);
        const int32_t px = (int32_t)bx + tx, py = (int32_t)by + ty;
        if (a1) body(PlanSrc<FP, RAW, STD, true>{t, tile, x0, y0, &P, &L, px, py});
        else body(PlanSrc<FP, RAW, STD, false>{t, tile, x0, y0, &P, &L, px, py});
        return;
    }
    const Span sx = tap_span(bx, min(bx + 15u, ow - 1u), Rw, k.du_min(), k.du_max(), t.w);
    const Span sy = tap_span(by, min(by + 15u, oh - 1u), Rh, k.dv_min(), k.dv_max(), t.h);
    if (sx.n <= FP && sy.n <= FP) {  // block-uniform
        // all of this thread's texel loads first, then the decodes (the loads' L2 latency overlaps)
        constexpr int R = (FP * FP + 255) / 256;
        uint32_t raw[R];
        const int32_t n = sx.n * sy.n;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int32_t i = (int32_t)threadIdx.x + r * 256;
            if (i < n) {
                const int32_t ly = i / sx.n, lx = i - ly * sx.n;
                raw[r] = t.px[(uint32_t)(sy.lo + ly) * t.w + (sx.lo + lx)];
            }
        }
        load_tables(tb, L);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int32_t i = (int32_t)threadIdx.x + r * 256;
            if (i < n) {
                const int32_t ly = i / sx.n, lx = i - ly * sx.n;
                const F4 d = dec(L, raw[r]);
                tile[ly * FP + lx] = make_float4(d.r, d.g, d.b, d.a);
            }
        }
        __syncthreads();
        body(TileSrc<FP>{t, tile, sx.lo, sy.lo});
    } else {
        load_tables(tb, L);
        body(GlobalSrc{t, &L});
    }
}

// occupancy floor for the 8-tap kernels: the unrolled taps otherwise take 160 VGPRs (3 waves/SIMD)
#define BLOOM_BOUNDS __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
constexpr int FP_UP = 24;     // staged footprint of a generic up pass (taps within a few texels)
constexpr int FP_Y = 24;      // blur1 at full size: taps within +-3 texels (22 x 22)
constexpr int FP_FINAL = 44;  // the last up pass at res / 4: taps within +-12 texels (42 x 42)

// ---- separable plan of an 8-tap pass (any frame size) -------------------------------------------
// A tap's texel coordinate along x depends only on the pixel's column (texcoord(x) + du_i, then
// sample_coord and floor), and along y only on its row.  The host evaluates that arithmetic once per
// launch shape for every column and row (bh_bloom_sep_plan: the kernel's own f32 operations, no
// contraction) and the kernel reads it instead of recomputing it per pixel: the general sampler's lerps
// on the general sampler's texels, the same bits.  Used by the up passes whose TapPlan / Up2Plan proofs
// fail (frame sizes other than powers of two).
// Entry per tap and column (then per tap and row): the UNCLAMPED floor f of the sampler's coordinate t
// (t clamped to [-1, n] as sample_coord does, so f is in [-1, n]) and the weights fa = t - f (in [0, 1]: a t just
// below an integer rounds t - f up to 1),
// ia = 1 - fa.  The block stages its footprint with clamp-to-edge addressing -- tile entry (ly, lx)
// holds texel (clamp(lo_y + ly), clamp(lo_x + lx)) -- so sample()'s texels clamp(f) and clamp(f + 1)
// are tile entries f - lo and f + 1 - lo: a tap's four reads are one base offset plus 0, 1, FP, FP + 1.
struct SepEntry { int32_t f; float fa, ia; int32_t pad; };
static_assert(sizeof(SepEntry) == 16, "one ds_read_b128 per entry");

// Epilogues of the separable up pass.  PLAIN: out = q(up8).  Y (the general fused chain's first stage,
// source X): U = q(up8(X)) to `aux` for every pixel, and Y = q(X + 0.5 U) to `out` for the pixels whose
// column and row sample exactly (same-size plan weight 0; the rest: fixup_kernel).  FINAL (source U0
// = the blur's last up input, res = res[L]): B = q(up8(U0)) to `aux`, and for exact pixels
// out = q(col + 0.5 q(Y + 0.5 B)) (own0 = col, own1 = Y).
enum SepEpi : uint32_t { EPI_PLAIN = 0, EPI_Y = 1, EPI_FINAL = 2 };

// bilinear of texels (t00, t10, t01, t11) with weights (fa, fb): sample()'s operations in its order
__device__ __forceinline__ F4 lerp_plan(const float4& t00, const float4& t10, const float4& t01, const float4& t11,
                                        float fa, float fb) {
    const float ia = 1.0f - fa, ib = 1.0f - fb;
    F4 q;
    q.r = (t00.x * ia + t10.x * fa) * ib + (t01.x * ia + t11.x * fa) * fb;
    q.g = (t00.y * ia + t10.y * fa) * ib + (t01.y * ia + t11.y * fa) * fb;
    q.b = (t00.z * ia + t10.z * fa) * ib + (t01.z * ia + t11.z * fa) * fb;
    q.a = (t00.w * ia + t10.w * fa) * ib + (t01.w * ia + t11.w * fa) * fb;
    return q;
}

// FP: the staged footprint's side.  RAW: the tile holds the BGRA8 words (4 B per texel instead of 16, for
// the wide footprint of the final pass: 44 x 48 words = 8.4 KiB instead of 33 KiB), decoded when a tap
// reads them.  FS: the tile's row stride, a multiple of 16 float4 for the decoded tile (ds_read_b128 lane
// groups take two rows: see FS_YQ; in a same-size pass lane l reads column ~l & 15 of row ~l >> 4) and 16
// mod 32 words for the raw one (ds_read_b32: lanes 0-15 row r, 16-31 row r + 1 land on the other banks).
template <int FP, bool RAW>
constexpr int sep_stride() { return RAW ? (FP + 16) / 32 * 32 + 16 : (FP + 15) / 16 * 16; }
template <int FP, uint32_t EPI, bool RAW = false, int FS = sep_stride<FP, RAW>()>
__global__ void BLOOM_BOUNDS up_sep_kernel(Tables tb, CTex a, uint32_t rx, uint32_t ry, const SepEntry* __restrict__ sep,
                                           Tex out, CTex own0, CTex own1, const uint2* __restrict__ same, Tex aux) {
    __shared__ Lds L;
    __shared__ std::conditional_t<RAW, uint32_t, float4> tile[FP * FS];
    __shared__ SepEntry colp[8][16], rowp[8][16];
    const uint32_t bx = xcd_block().x * 16u, by = xcd_block().y * 16u;
    const uint32_t ow = EPI == EPI_PLAIN ? out.w : aux.w, oh = EPI == EPI_PLAIN ? out.h : aux.h;
    const uint32_t tx = threadIdx.x & 15u, ty = threadIdx.x >> 4;
    const uint32_t x = bx + tx, y = by + ty;
    const bool in = x < ow && y < oh;
    // the block's footprint from the sampler's own arithmetic (no memory round trip before the staging
    // loads): every rounding step is monotone in the texcoord, so the extreme taps (du(0) and du(4), dv(6)
    // and dv(2)) of the first and last column (row) bound every tap's floor -- exactly the plan's extremes
    const crm::Rcp Rw = crm::rcp_refined((float)ow), Rh = crm::rcp_refined((float)oh);
    const Taps k(rx, ry);
    const uint32_t xl = min(bx + 15u, ow - 1u), yl = min(by + 15u, oh - 1u);
    const int32_t lo_x = (int32_t)floorf(sample_coord(texcoord(bx, Rw) + k.du_min(), a.w));
    const int32_t hi_x = (int32_t)floorf(sample_coord(texcoord(xl, Rw) + k.du_max(), a.w));
    const int32_t lo_y = (int32_t)floorf(sample_coord(texcoord(by, Rh) + k.dv_min(), a.h));
    const int32_t hi_y = (int32_t)floorf(sample_coord(texcoord(yl, Rh) + k.dv_max(), a.h));
    const int32_t cx = min(hi_x - lo_x + 2, FP), cy = min(hi_y - lo_y + 2, FP);  // floor .. floor + 1
    // the host sizes FP for the launch (bh_bloom_sep_plan's extent), so the min never cuts
    constexpr int R = (FP * FP + 255) / 256;
    uint32_t raw[R];
    const int32_t wm = (int32_t)a.w - 1, hm = (int32_t)a.h - 1;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int32_t i = (int32_t)threadIdx.x + r * 256, ly = i / cx, lx = i - ly * cx;
        raw[r] = 0xFF000000u;
        if (ly < cy) raw[r] = a.px[(uint32_t)clampi(lo_y + ly, 0, hm) * a.w + clampi(lo_x + lx, 0, wm)];
    }
    // this block's plan entries as tile offsets: thread t < 128 column entry (t >> 4, t & 15), else row
    {
        const uint32_t i = (threadIdx.x >> 4) & 7u, j = threadIdx.x & 15u;
        if (threadIdx.x < 128u) {
            SepEntry e = sep[i * ow + min(bx + j, ow - 1u)];
            e.f -= lo_x;
            colp[i][j] = e;
        } else {
            SepEntry e = sep[8u * ow + i * oh + min(by + j, oh - 1u)];
            e.f = (e.f - lo_y) * FS;
            rowp[i][j] = e;
        }
    }
    // own texels of the epilogue, loaded before the tables, used last
    const uint32_t pix = (in ? y : 0u) * ow + (in ? x : 0u);
    uint32_t o0 = 0xFF000000u, o1 = 0xFF000000u;
    bool exact = false;
    if constexpr (EPI != EPI_PLAIN) {
        o0 = own0.px[pix];
        if constexpr (EPI == EPI_FINAL) o1 = own1.px[pix];
        exact = in && same[in ? x : 0u].y == 0u && same[ow + (in ? y : 0u)].y == 0u;
    }
    load_tables(tb, L);  // after the footprint's loads are issued: both round trips overlap
    uint32_t m = min(o0, o1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int32_t i = (int32_t)threadIdx.x + r * 256, ly = i / cx, lx = i - ly * cx;
        if (ly < cy) {
            if constexpr (RAW) {
                tile[ly * FS + lx] = raw[r];
            } else {
                const F4 d = dec(L, raw[r]);
                tile[ly * FS + lx] = make_float4(d.r, d.g, d.b, d.a);
            }
        }
        m = min(m, raw[r]);
    }
    // every staged texel (and every own texel) opaque: alpha 1.0 throughout, its arithmetic folds away
    const bool a1 = barrier_and(m >= 0xFF000000u);
    if (!in) return;
    auto run = [&](auto A1c) {
        constexpr bool A1 = decltype(A1c)::value;
        F4 s{0.0f, 0.0f, 0.0f, 0.0f};
        SepEntry c = colp[0][tx], r = rowp[0][ty];
        // software-pipelined: tap i + 1's four tile reads are issued before tap i computes (the LDS
        // latency of one tap hides behind the other's lerps); RAW tiles pipeline the words, decoded at use
        using W = std::conditional_t<RAW, uint32_t, float4>;
        auto word = [&](int32_t o) -> W { return tile[o]; };
        W w00, w10, w01, w11;
        {
            const int32_t o = c.f + r.f;
            w00 = word(o); w10 = word(o + 1); w01 = word(o + FS); w11 = word(o + FS + 1);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            // the next tap's plan entries are read while this tap computes; one tap at a time otherwise
            // (the sched barrier and the empty asm on the sums keep the compiler from hoisting later taps'
            // texel reads or sinking this tap's work: all 8 together take ~160 VGPRs)
            SepEntry cn = c, rn = r;
            if (i < 7) {
                cn = colp[i + 1][tx];
                rn = rowp[i + 1][ty];
            }
            const W v00 = w00, v10 = w10, v01 = w01, v11 = w11;
            if (i < 7) {
                const int32_t on = cn.f + rn.f;
                w00 = word(on); w10 = word(on + 1); w01 = word(on + FS); w11 = word(on + FS + 1);
            }
            auto unpack = [&](const W& v) {
                if constexpr (RAW) {
                    const F4 d = dec<A1>(L, v);
                    return make_float4(d.r, d.g, d.b, d.a);
                } else {
                    return v;
                }
            };
            const float4 t00 = unpack(v00), t10 = unpack(v10), t01 = unpack(v01), t11 = unpack(v11);
            const float ia = c.ia, fa = c.fa, ib = r.ia, fb = r.fa;  // sample()'s operations in its order
            F4 q;
            q.r = (t00.x * ia + t10.x * fa) * ib + (t01.x * ia + t11.x * fa) * fb;
            q.g = (t00.y * ia + t10.y * fa) * ib + (t01.y * ia + t11.y * fa) * fb;
            q.b = (t00.z * ia + t10.z * fa) * ib + (t01.z * ia + t11.z * fa) * fb;
            // an opaque block's texels all have alpha 1.0, and then every tap's alpha is exactly 1.0:
            // RN(ia + fa) == 1 for fa in [0, 1) and ia = RN(1 - fa) (|ia + fa - 1| <= 2^-25), likewise along y
            q.a = A1 ? 1.0f : (t00.w * ia + t10.w * fa) * ib + (t01.w * ia + t11.w * fa) * fb;
            acc(s, q, i);
            asm volatile("" ::"v"(s.r), "v"(s.g), "v"(s.b), "v"(s.a));
            __builtin_amdgcn_sched_barrier(0);
            c = cn;
            r = rn;
        }
        const F4 u = div12(s);
        if constexpr (EPI == EPI_PLAIN) {
            out.px[pix] = enc(L, u);
        } else {
            const uint32_t ue = enc(L, u);
            aux.px[pix] = ue;
            if (exact) {
                const F4 uq = dec<A1>(L, ue);
                if constexpr (EPI == EPI_Y) {
                    out.px[pix] = enc(L, remix(dec<A1>(L, o0), uq));
                } else {
                    const F4 z = quant<A1>(L, remix(dec<A1>(L, o1), uq));
                    out.px[pix] = enc(L, remix(dec<A1>(L, o0), z));
                }
            }
        }
    };
    if (a1) run(std::true_type{});
    else run(std::false_type{});
}

// ---- the separable up pass with one 2x2 pixel quad per lane (32x32 pixels per block) -------------------
// Adjacent pixels' taps mostly share texels: in a same-size pass a tap's floor steps by one texel per
// pixel, in a 2:1 pass by 0 or 1 with the pixel's parity.  Per tap, when every lane of the wave has the
// same steps (dx between its two columns' floors, dy between its two rows'), with dx, dy in {0, 1}, the
// quad's texels are one (2 + dx) x (2 + dy) window: 4..9 tile reads for four pixels instead of 16 (the
// LDS bandwidth bound the one-pixel kernel measured, §7b).  Each pixel still runs sample()'s lerps on its
// own four texels with its own column and row weights, in the same order: the same bits.  A wave whose
// steps differ (an exceptional column or row, the frame edge) reads each pixel's four texels.
// Tile layout: entry (ly, lx) at ly * FS + lx + (ly >> 1) -- every row pair shifted by one entry, so rows
// two apart (a same-size pass's consecutive quad rows) are 2 FS + 1 entries apart and the next quad row
// reads the other bank parity (the yq tile's row-pair shift, see FS_YQ).  A row entry of the plan holds
// that row offset and (pad) the row ly itself: the row below is FS + (ly & 1) further.
// The block's plan entries in 8 bytes (floor offset and row as int16, fa; ia = 1 - fa recomputed, the host
// plan's own operation) -- 4 KiB less LDS per block than the 16-byte SepEntry.
struct QEntry { int16_t f, pad; float fa; };
__device__ __forceinline__ float q_ia(const QEntry& e) { return 1.0f - e.fa; }
__device__ __forceinline__ QEntry q_entry(int32_t f, int32_t pad, const SepEntry& e) {
    return {(int16_t)f, (int16_t)pad, e.fa};
}
// The raw 60-word tile's row stride (any stride keeps the quad rows' bank parity: the next quad row is
// 2 FS + 1 words further, an odd number).  64 instead of 80: 15 KiB of tile instead of 19
constexpr int SEPQ_FS60 = 64;
// an occupancy floor of 6 waves per EU for the quad kernel
#define SEPQ_BOUNDS __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6)))
template <int FP, bool RAW>
constexpr int sepq_stride() { return RAW ? (FP + 16) / 32 * 32 + 16 : (FP + 15) / 16 * 16; }
// FIX (EPI_Y only): the block also recomputes its inexact pixels whose same-size sample stays inside the
// block -- S(X) from the staged tile, S(U1) from the block's own U words exchanged through LDS after a
// barrier -- so the fix-up pass keeps only the columns and rows whose sample crosses a block edge (none for
// the grid origin the host picks, bh_bloom_same_plan_org).  org: the block grid's origin, blocks start at
// 32 k - (org & 0xFFFF) columns and 32 k - (org >> 16) rows (even offsets: a quad never straddles the frame
// edge).
// With EPI_FINAL (FIX2 below) the fix reaches two texels: out = remix(S(col), S(F)) with F = q(remix(S(Y),
// S(B))) at the sample's texels, each of them exact (F is then the exact epilogue's own z) or itself sampled
// -- B from the block's words, Y and col from the block's own words, all through LDS.  Its three barriers
// come after the taps, so the dead tile holds the B, Y and F words and the dead plan entries the col words.
constexpr uint32_t FIX_WORDS = 32u * 33u;  // one padded 32 x 32 array of words
// The epilogue's own texels are loaded after the tile is staged ("late"), so that the launch's first waves
// load only their footprints (its opening burst is HBM-bound) and the own texels arrive during the taps; the
// block's opaque test then covers the footprint only, and the epilogue decodes the own texels' alpha unless
// its wave's own texels are all opaque too.
// The footprint is staged row by row -- wave w loads tile rows w, w + 4, ... (two rows per wave-instruction
// when FP <= 32), lane = column -- so each load's address is one 24-bit multiply-add off a per-lane column and
// a per-round row, and an out-of-footprint lane stores into a spare tile slot instead of branching; where rows
// of FP lanes take fewer rounds (FP = 40: 7 instead of 10) the element index is split by the constant FP
// instead.
template <int FP, bool RAW, int FS>
constexpr bool sepq_fix2_fits() {
    return sizeof(std::conditional_t<RAW, uint32_t, float4>) * (FP * FS + FP / 2) >= 3u * FIX_WORDS * 4u;
}
template <int FP, uint32_t EPI, bool RAW, int FS = sepq_stride<FP, RAW>(), bool FIX = false>
__global__ void SEPQ_BOUNDS up_sepq_kernel(Tables tb, CTex a, uint32_t rx, uint32_t ry,
                                                      const SepEntry* __restrict__ sep, Tex out, CTex own0, CTex own1,
                                                      const uint2* __restrict__ same, Tex aux, uint32_t org,
                                                      const uint32_t* __restrict__ stc, uint32_t* __restrict__ strips,
                                                      uint32_t strip_w) {
    // FIX2: the final epilogue's fix (an instantiation whose tile cannot hold its words never takes it; the
    // host does not request it there, bh_bloom_sep_fix_ok)
    constexpr bool FIX1 = FIX && EPI == EPI_Y, FIX2 = FIX && EPI == EPI_FINAL && sepq_fix2_fits<FP, RAW, FS>();
    constexpr bool LATE = EPI != EPI_PLAIN && !FIX2;
    using TileT = std::conditional_t<RAW, uint32_t, float4>;
    __shared__ Lds L;
    // + 1: the spare slot of the row-wise staging's out-of-footprint lanes
    __shared__ __attribute__((aligned(16))) unsigned char tile_mem[sizeof(TileT) * (FP * FS + FP / 2 + 1)];
    TileT* const tile = reinterpret_cast<TileT*>(tile_mem);
    // plan entries by parity (even columns, then odd): a quad's two entries are consecutive 16-B slots across
    // the lanes instead of every second one (2-way bank conflicts)
    __shared__ __attribute__((aligned(16))) QEntry cr[2][8][2][16];
    auto& colp = cr[0];
    auto& rowp = cr[1];
    static_assert(sizeof(cr) >= 32u * 32u * 4u, "FIX2's col words");
    __shared__ uint32_t ublk[FIX1 ? 32 : 1][FIX1 ? 33 : 1];  // the block's U words (FIX1)
    __shared__ uint32_t okc[FIX2 ? 32 : 1], okr[FIX2 ? 32 : 1];  // FIX2: F of the block column / row computable
    // FIX2: the same-size plan entries of the block's columns and rows, staged with the footprint (in registers
    // across the taps they pushed the final pass past its 80 VGPRs into scratch)
    __shared__ uint2 sce[FIX2 ? 32 : 1], sre[FIX2 ? 32 : 1];
    // the block's first column / row (negative for the first block of a grid with an origin offset: wrapped,
    // so x < ow fails for the columns left of the frame) and the first ones inside the frame
    const uint32_t bx = xcd_block().x * 32u - (org & 0xFFFFu), by = xcd_block().y * 32u - (org >> 16);
    const uint32_t bxf = (int32_t)bx < 0 ? 0u : bx, byf = (int32_t)by < 0 ? 0u : by;
    const uint32_t ow = EPI == EPI_PLAIN ? out.w : aux.w, oh = EPI == EPI_PLAIN ? out.h : aux.h;
    const uint32_t qx = threadIdx.x & 15u, qy = threadIdx.x >> 4;
    const uint32_t x0 = bx + 2u * qx, y0 = by + 2u * qy;  // the quad's first pixel
    // the block's footprint from the sampler's own arithmetic (see up_sep_kernel)
    const crm::Rcp Rw = crm::rcp_refined((float)ow), Rh = crm::rcp_refined((float)oh);
    const Taps k(rx, ry);
    const uint32_t xl = min(bx + 31u, ow - 1u), yl = min(by + 31u, oh - 1u);
    const int32_t lo_x = (int32_t)floorf(sample_coord(texcoord(bxf, Rw) + k.du_min(), a.w));
    const int32_t hi_x = (int32_t)floorf(sample_coord(texcoord(xl, Rw) + k.du_max(), a.w));
    const int32_t lo_y = (int32_t)floorf(sample_coord(texcoord(byf, Rh) + k.dv_min(), a.h));
    const int32_t hi_y = (int32_t)floorf(sample_coord(texcoord(yl, Rh) + k.dv_max(), a.h));
    const int32_t cx = min(hi_x - lo_x + 2, FP), cy = min(hi_y - lo_y + 2, FP);  // the host sizes FP: no cut
    const int32_t wm = (int32_t)a.w - 1, hm = (int32_t)a.h - 1;
    // rows per wave-instruction and rounds; LIN: rows of FP elements (constant split) when that takes fewer rounds
    constexpr int RPI = FP > 32 ? 1 : 2, RR = (FP + 4 * RPI - 1) / (4 * RPI), RL = (FP * FP + 255) / 256;
    constexpr bool LIN = RL < RR;
    constexpr int R = LIN ? RL : RR;
    const int32_t ln = (int32_t)(threadIdx.x & 63u);
    const int32_t rlx = RPI == 1 ? ln : (ln & 31), rly0 = (int32_t)(threadIdx.x >> 6) * RPI + (RPI == 1 ? 0 : ln >> 5);
    const uint32_t rcol = (uint32_t)clampi(lo_x + rlx, 0, wm);
    const bool rcol_in = rlx < cx;
    // element (ly, lx) of round r
    auto rl_at = [&](int r, int32_t& ly, int32_t& lx) {
        if constexpr (LIN) {
            const uint32_t i = threadIdx.x + 256u * (uint32_t)r;
            ly = (int32_t)(i / (uint32_t)FP);
            lx = (int32_t)i - ly * FP;
        } else {
            ly = rly0 + 4 * RPI * r;
            lx = rlx;
        }
    };
    uint32_t raw[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int32_t ly, lx;
        rl_at(r, ly, lx);
        const uint32_t col = LIN ? (uint32_t)clampi(lo_x + lx, 0, wm) : rcol;
        raw[r] = a.px[__umul24((uint32_t)clampi(lo_y + ly, 0, hm), a.w) + col];  // clamped: always inside
    }
    // plan entries as tile offsets: entry e < 256 column (e >> 5, e & 31), else row
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t i = (threadIdx.x >> 5) & 7u, j = threadIdx.x & 31u;
        if (h == 0) {
            const SepEntry e = sep[i * ow + (uint32_t)clampi((int32_t)(bx + j), 0, (int32_t)ow - 1)];
            colp[i][j & 1u][j >> 1] = q_entry(e.f - lo_x, 0, e);
        } else {
            const SepEntry e = sep[8u * ow + i * oh + (uint32_t)clampi((int32_t)(by + j), 0, (int32_t)oh - 1)];
            const int32_t ly = e.f - lo_y;
            rowp[i][j & 1u][j >> 1] = q_entry(ly * FS + (ly >> 1), ly, e);
        }
    }
    if constexpr (FIX2) {  // every block column's and row's entry (clamped: one outside the frame is never read)
        if (threadIdx.x < 32u) sce[threadIdx.x] = same[clampi((int32_t)(bx + threadIdx.x), 0, (int32_t)ow - 1)];
        else if (threadIdx.x < 64u) sre[threadIdx.x - 32u] = same[ow + clampi((int32_t)(by + threadIdx.x - 32u), 0, (int32_t)oh - 1)];
    }
    // own texels of the epilogue (four pixels), loaded before the tables (LATE: after the staging), used last
    uint32_t o0[2][2], o1[2][2];
    bool in[2][2], exact[2][2];
    uint2 scx[2] = {}, scy[2] = {};  // same-size plan entries of the quad's columns and rows (FIX1)
    uint32_t m = 0xFF000000u;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint32_t x = x0 + c, y = y0 + b;
            in[b][c] = x < ow && y < oh;
            const uint32_t pix = (in[b][c] ? y : 0u) * ow + (in[b][c] ? x : 0u);
            o0[b][c] = o1[b][c] = 0xFF000000u;
            exact[b][c] = false;
            if constexpr (EPI != EPI_PLAIN) {
                if constexpr (!LATE) {
                    o0[b][c] = own0.px[pix];
                    if constexpr (EPI == EPI_FINAL) o1[b][c] = own1.px[pix];
                }
                if constexpr (FIX2) {
                    // exact[] after the staging barrier, from sce / sre
                } else if constexpr (FIX1) {
                    if (b == 0) scx[c] = same[in[b][c] ? x : 0u];
                    if (c == 0) scy[b] = same[ow + (in[b][c] ? y : 0u)];
                    exact[b][c] = in[b][c] && scx[c].y == 0u && scy[b].y == 0u;
                } else {
                    exact[b][c] = in[b][c] && same[in[b][c] ? x : 0u].y == 0u && same[ow + (in[b][c] ? y : 0u)].y == 0u;
                }
            }
            m = min(m, min(o0[b][c], o1[b][c]));
        }
    load_tables(tb, L);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int32_t ly, lx;
        rl_at(r, ly, lx);
        const bool v = (LIN ? lx < cx : rcol_in) && ly < cy;
        const int32_t o = v ? ly * FS + lx + (ly >> 1) : FP * FS + FP / 2;  // else the spare slot
        if constexpr (RAW) {
            tile[o] = raw[r];
        } else {
            const F4 d = dec(L, raw[r]);
            tile[o] = make_float4(d.r, d.g, d.b, d.a);
        }
        m = min(m, v ? raw[r] : 0xFF000000u);
    }
    const bool a1 = barrier_and(m >= 0xFF000000u);
    if constexpr (FIX2) {
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int c = 0; c < 2; ++c) exact[b][c] = in[b][c] && sce[2u * qx + c].y == 0u && sre[2u * qy + b].y == 0u;
    }
    if constexpr (LATE) {
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const uint32_t pix = (in[b][c] ? y0 + b : 0u) * ow + (in[b][c] ? x0 + c : 0u);
                o0[b][c] = own0.px[pix];
                if constexpr (EPI == EPI_FINAL) o1[b][c] = own1.px[pix];
            }
        __builtin_amdgcn_sched_barrier(0);  // issued here, awaited in the epilogue
    }
    // a quad whose first pixel is outside is outside as a whole (even origin offsets); it has no taps, but
    // with FIX its lanes still meet the block's barriers
    const bool live = in[0][0];
    uint32_t bw[2][2] = {}, fw[2][2] = {};  // FIX2: the quad's B words and (exact pixels) F words
    if (!FIX1 && !FIX2 && !live) return;
    {
    auto run = [&](auto A1c) {
        constexpr bool A1 = decltype(A1c)::value;
        auto texel = [&](int32_t o) {
            if constexpr (RAW) {
                const F4 d = dec<A1>(L, tile[o]);
                return make_float4(d.r, d.g, d.b, d.a);
            } else {
                const float4 v = tile[o];
                return make_float4(v.x, v.y, v.z, A1 ? 1.0f : v.w);
            }
        };
        auto lerp = [&](const float4& t00, const float4& t10, const float4& t01, const float4& t11, const QEntry& c,
                        const QEntry& r) {
            const float ia = q_ia(c), fa = c.fa, ib = q_ia(r), fb = r.fa;  // sample()'s operations in its order
            F4 q;
            q.r = (t00.x * ia + t10.x * fa) * ib + (t01.x * ia + t11.x * fa) * fb;
            q.g = (t00.y * ia + t10.y * fa) * ib + (t01.y * ia + t11.y * fa) * fb;
            q.b = (t00.z * ia + t10.z * fa) * ib + (t01.z * ia + t11.z * fa) * fb;
            q.a = A1 ? 1.0f : (t00.w * ia + t10.w * fa) * ib + (t01.w * ia + t11.w * fa) * fb;
            return q;
        };
        if (live) {
        F4 s[2][2];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const QEntry cL = colp[i][0][qx], cR = colp[i][1][qx];
            const QEntry rT = rowp[i][0][qy], rB = rowp[i][1][qy];
            const int32_t dx = cR.f - cL.f, dy = rB.pad - rT.pad;  // the two columns' / rows' floor steps
            const int32_t dx0 = __builtin_amdgcn_readfirstlane(dx), dy0 = __builtin_amdgcn_readfirstlane(dy);
            const bool ux = __builtin_amdgcn_ballot_w64(dx != dx0) == 0ull && (dx0 == 0 || dx0 == 1);
            const bool uy = __builtin_amdgcn_ballot_w64(dy != dy0) == 0ull && (dy0 == 0 || dy0 == 1);
            const bool uni = ux && uy;
            const int32_t o = cL.f + rT.f;
            const int32_t d1 = FS + (rT.pad & 1), d2 = 2 * FS + 1;  // the window's rows 1 and 2
            auto window = [&](auto DXc, auto DYc) {
                constexpr int DX = decltype(DXc)::value, DY = decltype(DYc)::value;
                // rows 0 and 1 for the top pixels, then row 2 replaces row 0 for the bottom ones: 2 (2 + DX)
                // texels live at a time instead of 3 (2 + DX)
                float4 t0[2 + DX], t1[2 + DX];
#pragma unroll
                for (int c = 0; c < 2 + DX; ++c) { t0[c] = texel(o + c); t1[c] = texel(o + d1 + c); }
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const int ca = c ? DX : 0;
                    acc(s[0][c], lerp(t0[ca], t0[ca + 1], t1[ca], t1[ca + 1], c ? cR : cL, rT), i);
                }
                if constexpr (DY == 1) {
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int c = 0; c < 2 + DX; ++c) t0[c] = texel(o + d2 + c);
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const int ca = c ? DX : 0;
                        acc(s[1][c], lerp(t1[ca], t1[ca + 1], t0[ca], t0[ca + 1], c ? cR : cL, rB), i);
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const int ca = c ? DX : 0;
                        acc(s[1][c], lerp(t0[ca], t0[ca + 1], t1[ca], t1[ca + 1], c ? cR : cL, rB), i);
                    }
                }
            };
            if (uni && dx0 == 1 && dy0 == 1) window(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
            else if (uni && dx0 == 0 && dy0 == 1) window(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
            else if (uni && dx0 == 1 && dy0 == 0) window(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
            else if (uni && dx0 == 0 && dy0 == 0) window(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
            else {
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const QEntry& ce = c ? cR : cL;
                        const QEntry& re = b ? rB : rT;
                        const int32_t op = ce.f + re.f, dn = FS + (re.pad & 1);
                        acc(s[b][c], lerp(texel(op), texel(op + 1), texel(op + dn), texel(op + dn + 1), ce, re), i);
                    }
            }
            asm volatile("" ::"v"(s[0][0].r), "v"(s[0][1].r), "v"(s[1][0].r), "v"(s[1][1].r));
            __builtin_amdgcn_sched_barrier(0);
        }
        // STRIPS (final epilogue, stc != null): the column strips of the fix-up pass -- each column within 2 of
        // an inexact column (stc: 1 + its strip column, bh_bloom_strip_table) also stores its col, Y and U
        // words column-major, (image * strip_w + strip column) * oh + row
        uint32_t st[2] = {0u, 0u};
        if constexpr (EPI == EPI_FINAL && !FIX2) {
            if (stc) {
                st[0] = stc[min(x0, ow - 1u)];
                st[1] = stc[min(x0 + 1u, ow - 1u)];
            }
        }
        // LATE: the own texels were not in the block's opaque test; AO: the wave's are opaque as well
        bool own_op = true;
        if constexpr (LATE && A1) {
            uint32_t mo = 0xFFFFFFFFu;
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int c = 0; c < 2; ++c) mo = min(mo, min(o0[b][c], o1[b][c]));
            own_op = __builtin_amdgcn_ballot_w64(mo < 0xFF000000u) == 0ull;
        }
        auto epilogue = [&](auto AOc) {
        constexpr bool AO = decltype(AOc)::value;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (!in[b][c]) continue;
                const uint32_t pix = (y0 + b) * ow + x0 + c;
                const F4 u = div12(s[b][c]);
                if constexpr (EPI == EPI_PLAIN) {
                    out.px[pix] = enc(L, u);
                } else {
                    const uint32_t ue = enc(L, u);
                    aux.px[pix] = ue;
                    if constexpr (EPI == EPI_FINAL && !FIX2) {
                        if (st[c] != 0u) {
                            const size_t img = (size_t)strip_w * oh;
                            uint32_t* const p = strips + (size_t)(st[c] - 1u) * oh + (y0 + b);
                            p[0] = o0[b][c];
                            p[img] = o1[b][c];
                            p[2u * img] = ue;
                        }
                    }
                    if constexpr (FIX1) ublk[2u * qy + b][2u * qx + c] = ue;
                    if constexpr (FIX2) bw[b][c] = ue;
                    if (exact[b][c]) {
                        const F4 uq = dec<AO>(L, ue);
                        if constexpr (EPI == EPI_Y) {
                            out.px[pix] = enc(L, remix(dec<AO>(L, o0[b][c]), uq));
                        } else {
                            // z = q(Y + 0.5 B): F at this exact pixel, kept as its word for FIX2
                            const uint32_t zq = enc(L, remix(dec<AO>(L, o1[b][c]), uq));
                            if constexpr (FIX2) fw[b][c] = zq;
                            out.px[pix] = enc(L, remix(dec<AO>(L, o0[b][c]), dec<AO>(L, zq)));
                        }
                    }
                }
            }
        };
        if (A1 && own_op) epilogue(std::bool_constant<A1>{});
        else epilogue(std::false_type{});
        }  // live
        if constexpr (FIX2) {
            // the taps of every wave are done: the tile and the plan entries are dead
            __syncthreads();
            scx[0] = sce[2u * qx]; scx[1] = sce[2u * qx + 1u];
            scy[0] = sre[2u * qy]; scy[1] = sre[2u * qy + 1u];
            uint32_t(*const ub)[33] = reinterpret_cast<uint32_t(*)[33]>(tile_mem);
            uint32_t(*const yb)[33] = ub + 32;
            uint32_t(*const fb_)[33] = ub + 64;
            uint32_t(*const cb)[32] = reinterpret_cast<uint32_t(*)[32]>(&cr[0][0][0][0]);
            // a block column's (row's) F is computable here when it is exact or its sample's texels lie in
            // the block (nonzero weights only)
            auto axis_ok = [&](uint2 e, int32_t b0) {
                if (e.y == 0u) return true;
                return (uint32_t)((int32_t)(e.x & 0xFFFFu) - b0) <= 31u && (uint32_t)((int32_t)(e.x >> 16) - b0) <= 31u;
            };
            if (live) {
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        if (!in[b][c]) continue;
                        const uint32_t py = 2u * qy + b, px = 2u * qx + c;
                        ub[py][px] = bw[b][c];
                        yb[py][px] = o1[b][c];
                        cb[py][px] = o0[b][c];
                        if (exact[b][c]) fb_[py][px] = fw[b][c];
                    }
            }
            // every lane, live or not: a block row (column) outside the frame still has in-frame columns (rows)
            if (qy == 0u) { okc[2u * qx] = axis_ok(scx[0], (int32_t)bx); okc[2u * qx + 1u] = axis_ok(scx[1], (int32_t)bx); }
            if (qx == 0u) { okr[2u * qy] = axis_ok(scy[0], (int32_t)by); okr[2u * qy + 1u] = axis_ok(scy[1], (int32_t)by); }
            __syncthreads();
            // the sample's block-relative texels of one axis (a weight-0 texel repeats the first: t * 0 == +0)
            auto texels = [&](uint2 e, int32_t b0, int32_t& t0, int32_t& t1, float& w) {
                w = __uint_as_float(e.y);
                t0 = (int32_t)(e.x & 0xFFFFu) - b0;
                t1 = w != 0.0f ? (int32_t)(e.x >> 16) - b0 : t0;
            };
            auto D = [&](uint32_t w) {
                const F4 d = dec<A1>(L, w);
                return make_float4(d.r, d.g, d.b, d.a);
            };
            // F = q(remix(S(Y), S(B))) at this lane's inexact pixels whose F is computable
            if (live) {
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        if (!in[b][c] || exact[b][c]) continue;
                        const uint32_t py = 2u * qy + b, px = 2u * qx + c;
                        if (okc[px] == 0u || okr[py] == 0u) continue;
                        int32_t u0, u1, v0, v1;
                        float fa, fb;
                        texels(scx[c], (int32_t)bx, u0, u1, fa);
                        texels(scy[b], (int32_t)by, v0, v1, fb);
                        const F4 sy = lerp_plan(D(yb[v0][u0]), D(yb[v0][u1]), D(yb[v1][u0]), D(yb[v1][u1]), fa, fb);
                        const F4 sb = lerp_plan(D(ub[v0][u0]), D(ub[v0][u1]), D(ub[v1][u0]), D(ub[v1][u1]), fa, fb);
                        fb_[py][px] = enc(L, remix(sy, sb));
                    }
            }
            __syncthreads();
            // out = remix(S(col), S(F)) at the inexact pixels whose sample's texels lie in the block and have
            // a computable F (fixup_gather_kernel<EPI_FINAL>'s arithmetic); the rest: the fix-up pass's
            if (live) {
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        if (!in[b][c] || exact[b][c]) continue;
                        int32_t u0, u1, v0, v1;
                        float fa, fb;
                        texels(scx[c], (int32_t)bx, u0, u1, fa);
                        texels(scy[b], (int32_t)by, v0, v1, fb);
                        if ((uint32_t)u0 > 31u || (uint32_t)u1 > 31u || (uint32_t)v0 > 31u || (uint32_t)v1 > 31u) continue;
                        if (okc[u0] == 0u || okc[u1] == 0u || okr[v0] == 0u || okr[v1] == 0u) continue;
                        const F4 sc = lerp_plan(D(cb[v0][u0]), D(cb[v0][u1]), D(cb[v1][u0]), D(cb[v1][u1]), fa, fb);
                        const F4 sf = lerp_plan(D(fb_[v0][u0]), D(fb_[v0][u1]), D(fb_[v1][u0]), D(fb_[v1][u1]), fa, fb);
                        out.px[(y0 + b) * ow + x0 + c] = enc(L, remix(sc, sf));
                    }
            }
        }
        if constexpr (FIX1) {
            // Y = remix(S(X), S(U1)) at the inexact pixels whose sample's texels (those of nonzero weight) lie
            // in this block: fixup_gather_kernel<EPI_Y>'s arithmetic, each texel from LDS (a texel of weight 0
            // enters the lerp as t * 0 == +0 for any finite t >= 0, as the fix-up's unread 0 does)
            __syncthreads();
            if (live) {
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        if (!in[b][c] || exact[b][c]) continue;
                        const uint2 ex = scx[c], ey = scy[b];
                        const float fa = __uint_as_float(ex.y), fb = __uint_as_float(ey.y);
                        const int32_t u0 = (int32_t)(ex.x & 0xFFFFu) - (int32_t)bx, v0 = (int32_t)(ey.x & 0xFFFFu) - (int32_t)by;
                        const int32_t u1 = fa != 0.0f ? (int32_t)(ex.x >> 16) - (int32_t)bx : u0;
                        const int32_t v1 = fb != 0.0f ? (int32_t)(ey.x >> 16) - (int32_t)by : v0;
                        if ((uint32_t)u0 > 31u || (uint32_t)u1 > 31u || (uint32_t)v0 > 31u || (uint32_t)v1 > 31u)
                            continue;  // crosses the block edge: the fix-up pass's (residual list)
                        auto X = [&](int32_t u, int32_t v) {
                            const int32_t ly = v + (int32_t)by - lo_y, lx = u + (int32_t)bx - lo_x;
                            return texel(ly * FS + lx + (ly >> 1));
                        };
                        auto U = [&](int32_t u, int32_t v) {
                            const F4 d = dec<A1>(L, ublk[v][u]);
                            return make_float4(d.r, d.g, d.b, d.a);
                        };
                        const F4 sx = lerp_plan(X(u0, v0), X(u1, v0), X(u0, v1), X(u1, v1), fa, fb);
                        const F4 su = lerp_plan(U(u0, v0), U(u1, v0), U(u0, v1), U(u1, v1), fa, fb);
                        out.px[(y0 + b) * ow + x0 + c] = enc(L, remix(sx, su));
                    }
            }
        }
    };
    if (a1) run(std::true_type{});
    else run(std::false_type{});
    }
}


// ---- remixes of the chain at any proven-identity size (general fused schedule) ----------------------
// On frames whose same-size passes are identities on stored texels (the host's same_size_identity, e.g.
// 1920x1080, 1280x720) the copies vanish, but a remix still SAMPLES its two inputs: at the few columns
// and rows where t = RN(RN((x + 0.5) / n) * n) - 0.5 misses x, the sample mixes in a neighbour with a tiny
// weight before the two samples are added, and that sum can round to another byte than the texels' sum.
// So these kernels sample every input through the same-size plan (bh_bloom_same_plan: per column and per
// row the two clamped texels and the weight, sample()'s own arithmetic) -- a pixel whose column and row
// are exact (weights 1 / 0) reads its own texel, which is that sample bit for bit.
// Plan layout: (x0 | x1 << 16, weight bits) per column [0, w), then per row [w, w + h).
template <bool A1 = false>
__device__ __forceinline__ F4 sample_same(const Lds& L, CTex t, uint2 cx, uint2 cy) {
    const int32_t x0 = (int32_t)(cx.x & 0xFFFFu), y0 = (int32_t)(cy.x & 0xFFFFu);
    const float fa = __uint_as_float(cx.y), fb = __uint_as_float(cy.y);
    const uint32_t r0 = (uint32_t)y0 * t.w;
    if (fa == 0.0f && fb == 0.0f) return dec<A1>(L, t.px[r0 + (uint32_t)x0]);
    const int32_t x1 = (int32_t)(cx.x >> 16), y1 = (int32_t)(cy.x >> 16);
    const uint32_t r1 = (uint32_t)y1 * t.w;
    const F4 a = dec<A1>(L, t.px[r0 + (uint32_t)x0]), b = dec<A1>(L, t.px[r0 + (uint32_t)x1]);
    const F4 c = dec<A1>(L, t.px[r1 + (uint32_t)x0]), d = dec<A1>(L, t.px[r1 + (uint32_t)x1]);
    return lerp_plan(make_float4(a.r, a.g, a.b, a.a), make_float4(b.r, b.g, b.b, b.a), make_float4(c.r, c.g, c.b, c.a),
                     make_float4(d.r, d.g, d.b, d.a), fa, fb);
}
// out = remix(A, B) (remix.wgsl:22-24) with both inputs sampled through the plan
__global__ void __launch_bounds__(256) remix_plan_kernel(Tables tb, CTex A, CTex B, const uint2* __restrict__ plan,
                                                         Tex out) {
    __shared__ Lds L;
    const uint32_t x = xcd_block().x * 16u + (threadIdx.x & 15u), y = xcd_block().y * 16u + (threadIdx.x >> 4);
    const bool in = x < out.w && y < out.h;
    const uint2 cx = plan[in ? x : 0u], cy = plan[out.w + (in ? y : 0u)];
    load_tables(tb, L);
    if (!in) return;
    out.px[y * out.w + x] = enc(L, remix(sample_same(L, A, cx, cy), sample_same(L, B, cx, cy)));
}
// The chain's last two remixes: out = remix(col, F), F = q(remix(Y, Bt)) -- F is a texture of the
// reference (final_in1), so where the plan samples F between texels the lane evaluates F at each texel
// it weighs (at most 4, each sampling Y and Bt through the plan again).
__global__ void __launch_bounds__(256) remix2_plan_kernel(Tables tb, CTex col, CTex Y, CTex Bt,
                                                          const uint2* __restrict__ plan, Tex out) {
    __shared__ Lds L;
    const uint32_t x = xcd_block().x * 16u + (threadIdx.x & 15u), y = xcd_block().y * 16u + (threadIdx.x >> 4);
    const bool in = x < out.w && y < out.h;
    const uint2 cx = plan[in ? x : 0u], cy = plan[out.w + (in ? y : 0u)];
    load_tables(tb, L);
    if (!in) return;
    auto F = [&](uint32_t u, uint32_t v) {  // texel (u, v) of final_in1, decoded
        const uint2 px = plan[u], py = plan[out.w + v];
        return quant(L, remix(sample_same(L, Y, px, py), sample_same(L, Bt, px, py)));
    };
    const float fa = __uint_as_float(cx.y), fb = __uint_as_float(cy.y);
    const uint32_t x0 = cx.x & 0xFFFFu, x1 = cx.x >> 16, y0 = cy.x & 0xFFFFu, y1 = cy.x >> 16;
    F4 f;
    if (fa == 0.0f && fb == 0.0f) {
        f = F(x0, y0);
    } else {
        // the lerp of sample(): a texel whose weight is 0 enters as t * 0 == 0 for any finite t >= 0,
        // so it is not evaluated
        const F4 z{0.0f, 0.0f, 0.0f, 0.0f};
        const bool ex = fa != 0.0f, ey = fb != 0.0f;
        const F4 a = F(x0, y0), b = ex ? F(x1, y0) : z, c = ey ? F(x0, y1) : z, d = ex && ey ? F(x1, y1) : z;
        f = lerp_plan(make_float4(a.r, a.g, a.b, a.a), make_float4(b.r, b.g, b.b, b.a), make_float4(c.r, c.g, c.b, c.a),
                      make_float4(d.r, d.g, d.b, d.a), fa, fb);
    }
    out.px[y * out.w + x] = enc(L, remix(sample_same(L, col, cx, cy), f));
}

// The pixels the fused epilogues of up_sep_kernel skip: every pixel of a column or row whose same-size
// sample is inexact.  `list` = the n_cols inexact columns, then the n_rows inexact rows; thread i
// covers pixel i of the columns' pixels (all rows), then of the rows' pixels (all columns but the
// listed ones).  EPI_Y: out = remix(S(A), S(B)) (A = X, B = U1); EPI_FINAL: out = remix(S(A), S(F)),
// F = q(remix(S(B), S(C))) (A = col, B = Y, C = B-texture) -- remix_plan_kernel's / remix2_plan_kernel's
// per-pixel arithmetic.
// A same-size sample's texel words, gathered before the block stages its tables: (x0, y0), (x1, y0),
// (x0, y1), (x1, y1).  A word whose weight is 0 is not read (0 instead): it enters sample_same's lerp as
// t * 0 == +0 for any finite decoded t >= 0, so finish_same gives sample_same's bits.
struct SameWords { uint32_t t[4]; float fa, fb; };
__device__ __forceinline__ SameWords gather_same(CTex t, uint2 cx, uint2 cy) {
    const uint32_t x0 = cx.x & 0xFFFFu, x1 = cx.x >> 16, r0 = (cy.x & 0xFFFFu) * t.w, r1 = (cy.x >> 16) * t.w;
    SameWords s;
    s.fa = __uint_as_float(cx.y);
    s.fb = __uint_as_float(cy.y);
    const bool ex = s.fa != 0.0f, ey = s.fb != 0.0f;
    s.t[0] = t.px[r0 + x0];
    s.t[1] = ex ? t.px[r0 + x1] : 0u;
    s.t[2] = ey ? t.px[r1 + x0] : 0u;
    s.t[3] = ex && ey ? t.px[r1 + x1] : 0u;
    return s;
}
// The same gather from a texture (rs = row stride, cs = 1, xb = 0) or from a column strip of the fix-up
// (rs = 1, cs = H, xb = the strip's first column; xm caps the column offset: 4 in a strip)
struct SrcImg { const uint32_t* px; uint32_t rs, cs, xm; int32_t xb; };
__device__ __forceinline__ SameWords gather_img(SrcImg t, uint2 cx, uint2 cy) {
    auto at = [&](uint32_t x, uint32_t r) { return min((uint32_t)((int32_t)x - t.xb), t.xm) * t.cs + r * t.rs; };
    const uint32_t x0 = cx.x & 0xFFFFu, x1 = cx.x >> 16, r0 = cy.x & 0xFFFFu, r1 = cy.x >> 16;
    SameWords s;
    s.fa = __uint_as_float(cx.y);
    s.fb = __uint_as_float(cy.y);
    const bool ex = s.fa != 0.0f, ey = s.fb != 0.0f;
    s.t[0] = t.px[at(x0, r0)];
    s.t[1] = ex ? t.px[at(x1, r0)] : 0u;
    s.t[2] = ey ? t.px[at(x0, r1)] : 0u;
    s.t[3] = ex && ey ? t.px[at(x1, r1)] : 0u;
    return s;
}
__device__ __forceinline__ F4 finish_same(const Lds& L, const SameWords& s) {
    if (s.fa == 0.0f && s.fb == 0.0f) return dec(L, s.t[0]);
    const F4 a = dec(L, s.t[0]), b = dec(L, s.t[1]), c = dec(L, s.t[2]), d = dec(L, s.t[3]);
    return lerp_plan(make_float4(a.r, a.g, a.b, a.a), make_float4(b.r, b.g, b.b, b.a), make_float4(c.r, c.g, c.b, c.a),
                     make_float4(d.r, d.g, d.b, d.a), s.fa, s.fb);
}
// The general chain's same-size copies where they are not identities (bh_host.cpp bloom_chain: the reference's
// copy pass and the blur's same-size down, both the texel-centre sample, sample_same's arithmetic through the
// same-size plan): out = q(S(src)).  An exact pixel's sample is its own texel, so only the inexact columns' and
// rows' pixels gather and encode.
// A block covers 64 x 32 pixels, 8 rows per thread: its table staging (3 KiB) is paid once per 2048 pixels.
constexpr uint32_t SAME_COPY_ROWS = 8u;
__global__ void __launch_bounds__(256) same_copy_kernel(Tables tb, CTex src, const uint2* __restrict__ plan, Tex out) {
    __shared__ Lds L;
    const uint32_t W = src.w, H = src.h;
    const uint2 blk = xcd_block();
    const uint32_t x = blk.x * 64u + (threadIdx.x & 63u), y0 = blk.y * (4u * SAME_COPY_ROWS) + (threadIdx.x >> 6);
    const bool xin = x < W;
    const uint2 cx = plan[xin ? x : 0u];
    // every row's own word and plan entry first (independent loads: an exact pixel needs nothing else) ...
    uint32_t own[SAME_COPY_ROWS];
    uint2 cy[SAME_COPY_ROWS];
#pragma unroll
    for (uint32_t k = 0; k < SAME_COPY_ROWS; ++k) {
        const uint32_t y = min(y0 + 4u * k, H - 1u);
        cy[k] = plan[W + y];
        own[k] = src.px[y * W + (xin ? x : 0u)];
    }
    // ... then the inexact pixels' sample words, all rows' at once
    SameWords a[SAME_COPY_ROWS];
#pragma unroll
    for (uint32_t k = 0; k < SAME_COPY_ROWS; ++k) {
        a[k] = SameWords{{own[k], 0u, 0u, 0u}, 0.0f, 0.0f};
        if (cx.y != 0u || cy[k].y != 0u) a[k] = gather_same(src, cx, cy[k]);
    }
    load_tables(tb, L);
    if (!xin) return;
#pragma unroll
    for (uint32_t k = 0; k < SAME_COPY_ROWS; ++k) {
        const uint32_t y = y0 + 4u * k;
        if (y >= H) break;
        // an exact sample is its own texel, and q(dec(t)) == t for every stored word (the sRGB and alpha round
        // trips, which same_size_identity's exact class checks too): the word itself
        const bool exact = cx.y == 0u && cy[k].y == 0u;
        out.px[y * W + x] = exact ? own[k] : enc(L, finish_same(L, a[k]));
    }
}

// The gather form: the kernel's global reads in two dependent round trips (the list entry, then the
// plan entries of the pixel's column and row and of their neighbours, then every texel word) with the
// tables' staging overlapping them, instead of five (tables, list, plan, F's plan entries, texels).  A
// same-size sample's texels are its pixel's own and one neighbour (t is within an ulp-sized offset of
// the pixel's index), so F's plan entries are among the three preloaded per axis; `pick` reads the plan
// for any other index.
// rec (the host's records of the list, fixup_records): per entry two uint4, the column (row) and the plan
// entries of it and of its two neighbours (clamped), so the pixel's column and row entries and F's
// neighbours arrive with the list entry -- one dependent round trip fewer than list, then plan.
// strips (EPI_FINAL, the full list with records): a column lane (one row of an inexact column x) reads its
// texels -- all in x's strip at their offset from x (strip_ok) -- from the strips the final up pass's epilogue
// wrote, column-major (a wave's 64 rows: 256 contiguous bytes per strip column), instead of the three
// row-major textures, where each lane's word is a cache line of its own.  The record's word 7 is 1 + x's strip
// column.
template <uint32_t EPI>
__global__ void __launch_bounds__(256) fixup_gather_kernel(Tables tb, CTex A, CTex B, CTex C,
                                                           const uint2* __restrict__ plan,
                                                           const uint32_t* __restrict__ list, uint32_t n_cols,
                                                           uint32_t n_rows, Tex out, const uint4* __restrict__ rec,
                                                           const uint32_t* __restrict__ strips, uint32_t strip_w) {
    __shared__ Lds L;
    const uint32_t W = out.w, H = out.h;
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x, nc = (uint64_t)n_cols * H;
    uint32_t x = 0u, y = 0u, qx = 0u;  // qx: a column lane's strip column (strips)
    bool live = true;
    uint2 cx, cy, PX[3], PY[3];
    if (rec) {
        uint32_t k = 0u;
        bool col = true;
        if (i < nc) {
            k = (uint32_t)(i / H);
            y = (uint32_t)(i % H);
        } else {
            const uint64_t j = i - nc;
            live = j < (uint64_t)n_rows * W;
            col = false;
            if (live) {
                k = n_cols + (uint32_t)(j / W);
                x = (uint32_t)(j % W);
            }
        }
        const uint4 r0 = rec[2u * k], r1 = rec[2u * k + 1u];
        const uint2 e0 = make_uint2(r0.y, r0.z), e1 = make_uint2(r0.w, r1.x), e2 = make_uint2(r1.y, r1.z);
        if (col) {
            x = r0.x;
            qx = r1.w - 1u;
            PX[0] = e0; PX[1] = e1; PX[2] = e2;
            const uint32_t yc = min(y, H - 1u);
            PY[1] = plan[W + yc];
            if constexpr (EPI == EPI_FINAL) {
                PY[0] = plan[W + (yc ? yc - 1u : 0u)];
                PY[2] = plan[W + min(yc + 1u, H - 1u)];
            }
        } else {
            y = r0.x;
            PY[0] = e0; PY[1] = e1; PY[2] = e2;
            const uint32_t xc = min(x, W - 1u);
            PX[1] = plan[xc];
            if constexpr (EPI == EPI_FINAL) {
                PX[0] = plan[xc ? xc - 1u : 0u];
                PX[2] = plan[min(xc + 1u, W - 1u)];
            }
        }
        live = live && x < W && y < H;  // defensive: a list entry outside the frame
        cx = PX[1];
        cy = PY[1];
        // a dead lane (past the list, or a row lane's defensive case) gathers at pixel (0, 0) with every neighbour
        // entry its own: the record it read (entry 0 for a lane past the list, a column record) must not leave a
        // column's entry among the row ones, whose texel indices would then index rows (round 6's memory fault
        // at 3996 x 495: tools/bloom_fixup_addr.cpp)
        if (!live) { x = y = 0u; cx = plan[0]; cy = plan[W]; PX[0] = PX[1] = PX[2] = cx; PY[0] = PY[1] = PY[2] = cy; }
    } else {
        if (i < nc) {
            x = list[i / H];
            y = (uint32_t)(i % H);
        } else {
            const uint64_t j = i - nc;
            live = j < (uint64_t)n_rows * W;
            if (live) {
                y = list[n_cols + j / W];
                x = (uint32_t)(j % W);
            }
        }
        live = live && x < W && y < H;  // defensive: a list entry outside the frame
        if (!live) x = y = 0u;
        cx = plan[x];
        cy = plan[W + y];
        if constexpr (EPI == EPI_FINAL) {
            PX[0] = plan[x ? x - 1u : 0u]; PX[1] = cx; PX[2] = plan[min(x + 1u, W - 1u)];
            PY[0] = plan[W + (y ? y - 1u : 0u)]; PY[1] = cy; PY[2] = plan[W + min(y + 1u, H - 1u)];
        }
    }
    if (i >= nc && cx.y != 0u) live = false;  // an inexact column: its pixels are the first part's
    const bool sl = EPI == EPI_FINAL && strips != nullptr && rec != nullptr && i < nc;  // a column lane on strips
    auto img = [&](CTex T, uint32_t im) -> SrcImg {
        if (sl) return {strips + (size_t)im * strip_w * H, 1u, H, strip_w - 1u, (int32_t)x - (int32_t)qx};
        return {T.px, W, 1u, 0xFFFFFFFFu, 0};
    };
    const SameWords a = EPI == EPI_FINAL ? gather_img(img(A, 0u), cx, cy) : gather_same(A, cx, cy);
    if constexpr (EPI == EPI_Y) {
        const SameWords b = gather_same(B, cx, cy);
        load_tables(tb, L);
        if (live) out.px[y * W + x] = enc(L, remix(finish_same(L, a), finish_same(L, b)));
    } else {
        auto pick = [&](uint32_t u, uint32_t c, const uint2(&P)[3], uint32_t base) -> uint2 {
            if (u == c) return P[1];
            if (u + 1u == c) return P[0];
            if (u == c + 1u) return P[2];
            return plan[base + u];
        };
        const float fa = __uint_as_float(cx.y), fb = __uint_as_float(cy.y);
        const bool ex = fa != 0.0f, ey = fb != 0.0f;
        const uint2 px0 = pick(cx.x & 0xFFFFu, x, PX, 0u), px1 = pick(cx.x >> 16, x, PX, 0u);
        const uint2 py0 = pick(cy.x & 0xFFFFu, y, PY, W), py1 = pick(cy.x >> 16, y, PY, W);
        // F at the (up to 4) texels of final_in1 the lerp weighs (remix2_plan_kernel)
        SameWords fbw[4] = {}, fcw[4] = {};
        const SrcImg IB = img(B, 1u), IC = img(C, 2u);
        fbw[0] = gather_img(IB, px0, py0);
        fcw[0] = gather_img(IC, px0, py0);
        if (ex) {
            fbw[1] = gather_img(IB, px1, py0);
            fcw[1] = gather_img(IC, px1, py0);
        }
        if (ey) {
            fbw[2] = gather_img(IB, px0, py1);
            fcw[2] = gather_img(IC, px0, py1);
        }
        if (ex && ey) {
            fbw[3] = gather_img(IB, px1, py1);
            fcw[3] = gather_img(IC, px1, py1);
        }
        load_tables(tb, L);
        if (live) {
            auto F = [&](int k) { return quant(L, remix(finish_same(L, fbw[k]), finish_same(L, fcw[k]))); };
            const F4 z{0.0f, 0.0f, 0.0f, 0.0f};
            const F4 f0 = F(0), f1 = ex ? F(1) : z, f2 = ey ? F(2) : z, f3 = ex && ey ? F(3) : z;
            const F4 f = lerp_plan(make_float4(f0.r, f0.g, f0.b, f0.a), make_float4(f1.r, f1.g, f1.b, f1.a),
                                   make_float4(f2.r, f2.g, f2.b, f2.a), make_float4(f3.r, f3.g, f3.b, f3.a), fa, fb);
            out.px[y * W + x] = enc(L, remix(finish_same(L, a), f));
        }
    }
}

template <uint32_t EPI>
__global__ void __launch_bounds__(256) fixup_kernel(Tables tb, CTex A, CTex B, CTex C, const uint2* __restrict__ plan,
                                                    const uint32_t* __restrict__ list, uint32_t n_cols, uint32_t n_rows,
                                                    Tex out) {
    __shared__ Lds L;
    load_tables(tb, L);
    const uint32_t W = out.w, H = out.h;
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x, nc = (uint64_t)n_cols * H;
    uint32_t x, y;
    if (i < nc) {
        x = list[i / H];
        y = (uint32_t)(i % H);
    } else {
        const uint64_t j = i - nc;
        if (j >= (uint64_t)n_rows * W) return;
        y = list[n_cols + j / W];
        x = (uint32_t)(j % W);
        if (plan[x].y != 0u) return;  // an inexact column: its pixels are the first part's
    }
    if (x >= W || y >= H) return;  // defensive: a list entry outside the frame
    const uint2 cx = plan[x], cy = plan[W + y];
    if constexpr (EPI == EPI_Y) {
        out.px[y * W + x] = enc(L, remix(sample_same(L, A, cx, cy), sample_same(L, B, cx, cy)));
    } else {
        auto F = [&](uint32_t u, uint32_t v) {
            const uint2 px = plan[u], py = plan[W + v];
            return quant(L, remix(sample_same(L, B, px, py), sample_same(L, C, px, py)));
        };
        const float fa = __uint_as_float(cx.y), fb = __uint_as_float(cy.y);
        const uint32_t x0 = cx.x & 0xFFFFu, x1 = cx.x >> 16, y0 = cy.x & 0xFFFFu, y1 = cy.x >> 16;
        const F4 z{0.0f, 0.0f, 0.0f, 0.0f};
        const bool ex = fa != 0.0f, ey = fb != 0.0f;
        const F4 a = F(x0, y0), b = ex ? F(x1, y0) : z, c = ey ? F(x0, y1) : z, d = ex && ey ? F(x1, y1) : z;
        const F4 f = lerp_plan(make_float4(a.r, a.g, a.b, a.a), make_float4(b.r, b.g, b.b, b.a),
                               make_float4(c.r, c.g, c.b, c.a), make_float4(d.r, d.g, d.b, d.a), fa, fb);
        out.px[y * W + x] = enc(L, remix(sample_same(L, A, cx, cy), f));
    }
}

// One render pass of the reference (literal schedule): 16x16 pixels per 256-thread block.
template <uint32_t SH>
__global__ void BLOOM_BOUNDS pass_kernel(Tables tb, CTex a, CTex b, uint32_t rx, uint32_t ry, uint32_t point, TapPlan P,
                                        Tex out) {
    __shared__ Lds L;
    __shared__ float4 tile[SH == SH_UP ? FP_UP * FP_UP : 1];
    const uint32_t x = xcd_block().x * 16u + (threadIdx.x & 15u), y = xcd_block().y * 16u + (threadIdx.x >> 4);
    const crm::Rcp Rw = crm::rcp_refined((float)out.w), Rh = crm::rcp_refined((float)out.h);
    if constexpr (SH == SH_UP) {
        const Taps k(rx, ry);
        with_source<FP_UP>(tb, a, L, tile, k, out.w, out.h, Rw, Rh, P, [&](const auto& src) {
            if (x >= out.w || y >= out.h) return;
            out.px[(uint32_t)y * out.w + x] = enc(L, up8(src, k, texcoord(x, Rw), texcoord(y, Rh), point));
        });
    } else {
        // The sample's texel coordinates and weights (sample()'s own arithmetic).  Most pixels of a
        // same-size pass sample a texel centre (weights 0: the sample is that texel, sample_point),
        // and a 2:1 downsample the middle of 4 texels (weights 1/2: the exact quad form of TapPlan);
        // those take short forms, the others the general sampler -- the same bits either way.
        const bool in = x < out.w && y < out.h;
        const float u = texcoord(in ? x : 0u, Rw), v = texcoord(in ? y : 0u, Rh);
        const float tx = sample_coord(u, a.w), ty = sample_coord(v, a.h);
        const float fx = floorf(tx), fy = floorf(ty);
        const float fa = tx - fx, fb = ty - fy;
        const int32_t wm = (int32_t)a.w - 1, hm = (int32_t)a.h - 1;
        const int32_t x0 = clampi((int32_t)fx, 0, wm), y0 = clampi((int32_t)fy, 0, hm);
        const int32_t x1 = clampi((int32_t)fx + 1, 0, wm), y1 = clampi((int32_t)fy + 1, 0, hm);
        const bool centre = fa == 0.0f && fb == 0.0f;
        if constexpr (SH == SH_COPY || SH == SH_DOWN) {
            // a copy of a texel centre stores the texel's own word: enc(dec(t)) == t for every BGRA8 word
            // (sRGB: every code's decode encodes back to it; alpha: unorm8(k/255) == k --
            // tests/test_oracle.py::test_srgb_round_trip), so a block of centres needs no tables
            if (barrier_and(!in || centre)) {
                if (in) out.px[(uint32_t)y * out.w + x] = a.px[(uint32_t)y0 * a.w + (uint32_t)x0];
                return;
            }
        }
        load_tables(tb, L);
        if (!in) return;
        const GlobalSrc A{a, &L};
        F4 r;
        if constexpr (SH == SH_COPY || SH == SH_DOWN) {
            if (centre) {
                out.px[(uint32_t)y * out.w + x] = a.px[(uint32_t)y0 * a.w + (uint32_t)x0];
                return;
            }
            if (fa == 0.5f && fb == 0.5f) {
                // (t * 1/2 + t' * 1/2) == (t + t') * 1/2 for decoded texels, twice: ((t00 + t10) + (t01 + t11)) / 4
                const F4 q00 = A.at(x0, y0), q10 = A.at(x1, y0), q01 = A.at(x0, y1), q11 = A.at(x1, y1);
                r = {((q00.r + q10.r) + (q01.r + q11.r)) * 0.25f, ((q00.g + q10.g) + (q01.g + q11.g)) * 0.25f,
                     ((q00.b + q10.b) + (q01.b + q11.b)) * 0.25f, ((q00.a + q10.a) + (q01.a + q11.a)) * 0.25f};
            } else {
                r = sample(A, u, v);
            }
        } else {
            const GlobalSrc B{b, &L};
            if (centre) r = remix(A.at(x0, y0), B.at(x0, y0));
            else r = remix(sample(A, u, v), sample(B, u, v));
        }
        out.px[(uint32_t)y * out.w + x] = enc(L, r);
    }
}

// Two downsamples in one pass (the fused chains' blur: the intermediate level is read by nothing but the
// next downsample).  A texel of the intermediate level is pass_kernel<SH_DOWN>'s stored word at that
// pixel -- its arithmetic and its short forms, a centre's own word included -- and down2_kernel evaluates
// pass_kernel<SH_DOWN> over that texture, each texel it weighs computed on the spot.  A 2:1 downsample
// weighs each intermediate texel for one output pixel, so nothing is computed twice; the intermediate
// level is never stored.  Every texel index is arithmetic on the pixel's coordinates, so the 16 source
// words are read at once, before the block stages its tables (one dependent round trip, not three).
struct DownAt {  // the sampler's texels and weights of a pass pixel (sample()'s own arithmetic)
    int32_t x0, x1, y0, y1;
    float fa, fb;
};
__device__ __forceinline__ DownAt down_at(uint32_t x, uint32_t y, const crm::Rcp& Rw, const crm::Rcp& Rh, uint32_t sw,
                                          uint32_t sh) {
    const float u = texcoord(x, Rw), v = texcoord(y, Rh);
    const float tx = sample_coord(u, sw), ty = sample_coord(v, sh);
    const float fx = floorf(tx), fy = floorf(ty);
    const int32_t wm = (int32_t)sw - 1, hm = (int32_t)sh - 1;
    return {clampi((int32_t)fx, 0, wm), clampi((int32_t)fx + 1, 0, wm), clampi((int32_t)fy, 0, hm),
            clampi((int32_t)fy + 1, 0, hm), tx - fx, ty - fy};
}
// pass_kernel<SH_DOWN>'s value at a pixel from its four texels' words w (00, 10, 01, 11): the centre's own
// word (as a decoded value: enc(dec(t)) == t), the 2:1 quad form or sample()'s lerps
__device__ __forceinline__ F4 down_value(const Lds& L, const uint32_t (&w)[4], float fa, float fb) {
    const F4 q00 = dec(L, w[0]);
    if (fa == 0.0f && fb == 0.0f) return q00;
    const F4 q10 = dec(L, w[1]), q01 = dec(L, w[2]), q11 = dec(L, w[3]);
    F4 r;
    if (fa == 0.5f && fb == 0.5f) {
        r = {((q00.r + q10.r) + (q01.r + q11.r)) * 0.25f, ((q00.g + q10.g) + (q01.g + q11.g)) * 0.25f,
             ((q00.b + q10.b) + (q01.b + q11.b)) * 0.25f, ((q00.a + q10.a) + (q01.a + q11.a)) * 0.25f};
    } else {
        const float ia = 1.0f - fa, ib = 1.0f - fb;
        r.r = (q00.r * ia + q10.r * fa) * ib + (q01.r * ia + q11.r * fa) * fb;
        r.g = (q00.g * ia + q10.g * fa) * ib + (q01.g * ia + q11.g * fa) * fb;
        r.b = (q00.b * ia + q10.b * fa) * ib + (q01.b * ia + q11.b * fa) * fb;
        r.a = (q00.a * ia + q10.a * fa) * ib + (q01.a * ia + q11.a * fa) * fb;
    }
    return r;
}
// the stored word of a pass pixel: its centre's own word, else enc of the value
__device__ __forceinline__ uint32_t down_store(const Lds& L, const uint32_t (&w)[4], float fa, float fb) {
    return fa == 0.0f && fb == 0.0f ? w[0] : enc(L, down_value(L, w, fa, fb));
}
__global__ void BLOOM_BOUNDS down2_kernel(Tables tb, CTex a, uint32_t mw, uint32_t mh, Tex out) {
    __shared__ Lds L;
    const uint32_t x = xcd_block().x * 16u + (threadIdx.x & 15u), y = xcd_block().y * 16u + (threadIdx.x >> 4);
    const bool in = x < out.w && y < out.h;
    const DownAt o = down_at(in ? x : 0u, in ? y : 0u, crm::rcp_refined((float)out.w), crm::rcp_refined((float)out.h),
                             mw, mh);
    const crm::Rcp Mw = crm::rcp_refined((float)mw), Mh = crm::rcp_refined((float)mh);
    // the four intermediate texels (00, 10, 01, 11) and the four source words of each
    DownAt m[4];
    uint32_t w[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        m[k] = down_at((uint32_t)(k & 1 ? o.x1 : o.x0), (uint32_t)(k & 2 ? o.y1 : o.y0), Mw, Mh, a.w, a.h);
        const uint32_t r0 = (uint32_t)m[k].y0 * a.w, r1 = (uint32_t)m[k].y1 * a.w;
        w[k][0] = a.px[r0 + (uint32_t)m[k].x0];
        w[k][1] = a.px[r0 + (uint32_t)m[k].x1];
        w[k][2] = a.px[r1 + (uint32_t)m[k].x0];
        w[k][3] = a.px[r1 + (uint32_t)m[k].x1];
    }
    load_tables(tb, L);
    if (!in) return;
    uint32_t mid[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) mid[k] = down_store(L, w[k], m[k].fa, m[k].fb);
    out.px[y * out.w + x] = down_store(L, mid, o.fa, o.fb);
}

// Fused stage 1 (same-size sampling exact): Y = X + 0.5 * q(blur1(X)), blur1 = up8(X, res (W, H)).
__global__ void BLOOM_BOUNDS bloom_y_kernel(Tables tb, CTex X, uint32_t point, TapPlan P, Tex Y) {
    __shared__ Lds L;
    __shared__ float4 tile[FP_Y * FP_Y];
    const uint32_t x = xcd_block().x * 16u + (threadIdx.x & 15u), y = xcd_block().y * 16u + (threadIdx.x >> 4);
    const crm::Rcp Rw = crm::rcp_refined((float)Y.w), Rh = crm::rcp_refined((float)Y.h);
    const Taps k(X.w, X.h);
    with_source<FP_Y>(tb, X, L, tile, k, Y.w, Y.h, Rw, Rh, P, [&](const auto& src) {
        if (x >= Y.w || y >= Y.h) return;
        const F4 b1 = quant(L, up8(src, k, texcoord(x, Rw), texcoord(y, Rh), point));
        Y.px[(uint32_t)y * Y.w + x] = enc(L, remix(src.at((int32_t)x, (int32_t)y), b1));
    });
}

// Y in the TapPlan form with one 2x2 pixel quad per lane (32x32 pixels per block): per tap the quad's
// texels lie in a (2 + hx) x (2 + hy) neighbourhood at the plan's constant offset, read once for the
// four pixels (14 LDS reads per pixel instead of 21 at 4096x2048), each pixel reduced exactly as
// up8(PlanSrc) does.  HX / HY: the tap's half flags.
constexpr int FP_YQ = 40;  // 32 + the taps' reach (38 at 4096x2048)
// The tile's layout: entry (ly, lx) at ly * FS_YQ + lx + ((ly + p) >> 1), p = lo_y & 1 -- every second row
// pair shifted by one float4.  The quad loops' ds_read_b128 lane groups ({0-3, 12-15, 20-27}, {4-11, 16-19,
// 28-31}, ...: 16 lanes, one pass over the 64 banks) take two quad rows each, and a lane reads at quad
// column 2 (l & 15) -- only the even 4-bank slots of its quad row.  Without the shift the next quad row (two
// texel rows down) lands on the even slots too, whatever the row stride: 2-way conflicts (rocprofv3:
// SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 0.34 at strides 40 and 41).  With it a quad row is 2 FS_YQ + 1
// float4 further, odd: the next quad row reads the odd slots.  (p makes the quad's first texel row even in
// the shifted index, so a tap's row offsets are launch constants: yq_rowoff(d) = d FS_YQ + floor(d / 2).)
constexpr int FS_YQ = 40;
__host__ __device__ constexpr int32_t yq_rowoff(int32_t d) { return d * FS_YQ + (d >= 0 ? d / 2 : -((1 - d) / 2)); }
template <int HX, int HY>
__device__ __forceinline__ void yquad_tap(const float4* T, int32_t d1, int i, F4 (&s)[2][2]) {
    // T: the tap's first texel; the rows below it are d1 (FS_YQ or FS_YQ + 1) and 2 FS_YQ + 1 further
    float4 t[2 + HY][2 + HX];
#pragma unroll
    for (int r = 0; r < 2 + HY; ++r)
#pragma unroll
        for (int c = 0; c < 2 + HX; ++c) t[r][c] = T[(r == 0 ? 0 : r == 1 ? d1 : 2 * FS_YQ + 1) + c];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            float4 q = t[b][a];
            if constexpr (HX && HY) {
                const float4 u = t[b][a + 1], v = t[b + 1][a], w = t[b + 1][a + 1];
                q = make_float4((q.x + u.x) + (v.x + w.x), (q.y + u.y) + (v.y + w.y), (q.z + u.z) + (v.z + w.z),
                                (q.w + u.w) + (v.w + w.w));
            } else if constexpr (HX || HY) {
                const float4 u = HX ? t[b][a + 1] : t[b + 1][a];
                q = make_float4(q.x + u.x, q.y + u.y, q.z + u.z, q.w + u.w);
            }
            acc_scaled(s[b][a], q, HX + HY, i);
        }
}
// D2: the chain's next pass too, down2_kernel's two 2:1 downsamples of Y (bh_bloom_down2_fusable: frame sides
// multiples of 32, every sample of both levels the 0.5 / 0.5 average of the 2x2 texels below it): a lane's quad
// is the intermediate texel (x / 2, y / 2)'s four words, and four neighbouring lanes' intermediate words are the
// output pixel (x / 4, y / 4)'s -- down_store's arithmetic on the same words in the same order, so the same bits,
// and Y is not read back from memory.
template <int STD, bool D2 = false>
__global__ void BLOOM_BOUNDS bloom_yq_kernel(Tables tb, CTex X, TapPlan P, Tex Y, Tex D2o) {
    __shared__ Lds L;
    __shared__ float4 tile[FP_YQ * FS_YQ + FP_YQ / 2 + 1];
    const uint32_t bx = xcd_block().x * 32u, by = xcd_block().y * 32u;
    const int32_t x0 = (int32_t)bx + P.lo_x, y0 = (int32_t)by + P.lo_y;  // the footprint, clamp-to-edge
    const int32_t p = P.lo_y & 1;  // the row-pair shift's phase (see FS_YQ)
    {
        const int32_t nx = P.hi_x - P.lo_x + 32, ny = P.hi_y - P.lo_y + 32;
        const int32_t wm = (int32_t)X.w - 1, hm = (int32_t)X.h - 1;
        constexpr int R = (FP_YQ * FP_YQ + 255) / 256;
        uint32_t raw[R];
        // rows of FP_YQ elements (a constant split, see up_sepq_kernel's row-wise staging); the elements past the
        // footprint load clamped texels and store into the spare slot
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t i = threadIdx.x + 256u * (uint32_t)r;
            const int32_t ly = (int32_t)(i / (uint32_t)FP_YQ), lx = (int32_t)i - ly * FP_YQ;
            raw[r] = X.px[__umul24((uint32_t)clampi(y0 + ly, 0, hm), X.w) + (uint32_t)clampi(x0 + lx, 0, wm)];
        }
        load_tables(tb, L);  // after the footprint's loads are issued: both round trips overlap
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t i = threadIdx.x + 256u * (uint32_t)r;
            const int32_t ly = (int32_t)(i / (uint32_t)FP_YQ), lx = (int32_t)i - ly * FP_YQ;
            const bool v = lx < nx && ly < ny;
            const F4 d = dec(L, raw[r]);
            tile[v ? ly * FS_YQ + lx + ((ly + p) >> 1) : FP_YQ * FS_YQ + FP_YQ / 2] = make_float4(d.r, d.g, d.b, d.a);
        }
    }
    __syncthreads();
    const uint32_t x = bx + 2u * (threadIdx.x & 15u), y = by + 2u * (threadIdx.x >> 4);  // the quad's corner
    if (x >= Y.w || y >= Y.h) return;
    const int32_t m = (int32_t)y - y0;  // m + p is even
    const int32_t base = m * FS_YQ + ((m + p) >> 1) + ((int32_t)x - x0);
    F4 s[2][2];
    // Y = X + 0.5 q(blur1 / 12) per pixel of the quad; both pixels of each quad row in one 8-byte store:
    // inside the frame, and rows 8-byte aligned (even width; x is even); else one word per pixel
    auto finish = [&]() {
        const bool full = x + 1u < Y.w && y + 1u < Y.h && (Y.w & 1u) == 0u;
        uint32_t q[4];  // the quad's words: (x, y), (x + 1, y), (x, y + 1), (x + 1, y + 1)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            uint32_t c[2];
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const F4 b1 = quant(L, div12(s[b][a]));
                const float4 v = tile[base + b * FS_YQ + a];  // the pixel's own texel (row m + b, b < 2: no shift)
                c[a] = enc(L, remix({v.x, v.y, v.z, v.w}, b1));
                q[2 * b + a] = c[a];
            }
            if (full) {
                *reinterpret_cast<uint2*>(Y.px + (uint32_t)(y + b) * Y.w + x) = make_uint2(c[0], c[1]);
            } else {
#pragma unroll
                for (int a = 0; a < 2; ++a)
                    if (x + a < Y.w && y + b < Y.h) Y.px[(uint32_t)(y + b) * Y.w + x + a] = c[a];
            }
        }
        if constexpr (D2) {
            // every lane of the block is inside the frame (sides multiples of 32): the lane exchanges are complete
            const uint32_t mid = enc(L, down_value(L, q, 0.5f, 0.5f));  // the intermediate texel (x / 2, y / 2)
            const int l = (int)(threadIdx.x & 63u);
            const uint32_t w[4] = {mid, (uint32_t)__shfl_xor((int)mid, 1), (uint32_t)__shfl_xor((int)mid, 16),
                                   (uint32_t)__shfl_xor((int)mid, 17)};
            if ((l & 17) == 0)  // the lane of the 2x2 lane group's first quad: (x, y) multiples of 4
                D2o.px[(y >> 2) * D2o.w + (x >> 2)] = enc(L, down_value(L, w, 0.5f, 0.5f));
        }
    };
    if constexpr (STD != 0) {
        // the standard plan: constant offsets and halves, one tap at a time (see quad_taps_std)
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int32_t dy = fdiv8(STD * tap_m(1, i));
            const float4* T = tile + (base + yq_rowoff(dy) + fdiv8(STD * tap_m(0, i)));
            const int32_t d1 = yq_rowoff(dy + 1) - yq_rowoff(dy);
            switch ((fmod8(STD * tap_m(0, i)) == 4 ? 1 : 0) | (fmod8(STD * tap_m(1, i)) == 4 ? 2 : 0)) {
                case 0: yquad_tap<0, 0>(T, d1, i, s); break;
                case 1: yquad_tap<1, 0>(T, d1, i, s); break;
                case 2: yquad_tap<0, 1>(T, d1, i, s); break;
                default: yquad_tap<1, 1>(T, d1, i, s); break;
            }
            pin(s);
            __builtin_amdgcn_sched_barrier(0);
        }
        finish();
    } else {
#pragma unroll 1
        for (int i = 0; i < 8; i++) {
            const float4* T = tile + (base + yq_rowoff(P.oy[i]) + P.ox[i]);
            const int32_t d1 = FS_YQ + (P.oy[i] & 1);  // yq_rowoff(oy + 1) - yq_rowoff(oy)
            switch (((P.hx >> i) & 1u) | ((P.hy >> i) & 1u) << 1) {  // launch-uniform
                case 0: yquad_tap<0, 0>(T, d1, i, s); break;
                case 1: yquad_tap<1, 0>(T, d1, i, s); break;
                case 2: yquad_tap<0, 1>(T, d1, i, s); break;
                default: yquad_tap<1, 1>(T, d1, i, s); break;
            }
        }
        finish();
    }
}

// Fused last stage: out = col + 0.5 * q(Z), Z = Y + 0.5 * q(up8(U0, res (rx, ry))).
template <int STD>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) bloom_final_kernel(Tables tb, CTex col, CTex Y, CTex U0, uint32_t rx,
                                                   uint32_t ry, uint32_t point, TapPlan P, Tex out) {
    __shared__ Lds L;
    // dynamic: FP_FINAL^2 BGRA8 words for the TapPlan form (7.6 KiB: ~2x the resident blocks of the
    // decoded form, for a pass that mostly waits on its staging loads), else FP_FINAL^2 float4
    extern __shared__ float4 tile[];
    const uint32_t x = xcd_block().x * 16u + (threadIdx.x & 15u), y = xcd_block().y * 16u + (threadIdx.x >> 4);
    const crm::Rcp Rw = crm::rcp_refined((float)out.w), Rh = crm::rcp_refined((float)out.h);
    const Taps k(rx, ry);
    const bool in = x < out.w && y < out.h;
    const uint32_t i = (uint32_t)y * out.w + x;
    // the pixel's own Y and col texels: loaded after the footprint is staged (see up_sepq_kernel's LATE), in
    // flight during the taps; the block's opaque test covers the footprint, the wave's own texels pick the
    // last stage's form
    with_source<FP_FINAL, true, STD>(
        tb, U0, L, tile, k, out.w, out.h, Rw, Rh, P,
        [&](const auto& src) {
            constexpr bool A1 = std::decay_t<decltype(src)>::kA1;
            const uint32_t yv = in ? Y.px[i] : 0xFF000000u, cv = in ? col.px[i] : 0xFF000000u;
            __builtin_amdgcn_sched_barrier(0);
            if (!in) return;
            const F4 b3 = quant<A1>(L, up8(src, k, texcoord(x, Rw), texcoord(y, Rh), point));
            bool own_op = true;
            if constexpr (A1) own_op = __builtin_amdgcn_ballot_w64(min(yv, cv) < 0xFF000000u) == 0ull;
            auto fin = [&](auto AOc) {
                constexpr bool AO = decltype(AOc)::value;
                const F4 z = quant<AO>(L, remix(dec<AO>(L, yv), b3));
                out.px[i] = enc(L, remix(dec<AO>(L, cv), z));
            };
            if (A1 && own_op) fin(std::bool_constant<A1>{});
            else fin(std::false_type{});
        },
        true);
}

// ---- persistent blocks (standard plans) ------------------------------------------------------------
// The grid is the resident block count (a multiple of 8); block b walks the 16x16 tiles of one eighth of
// the frame (b % 8: the blocks the dispatcher deals to one XCD, whose L2 then holds the halos its tiles
// share) with stride gridDim / 8.  While a tile is computed from one LDS buffer, the next tile's
// footprint streams into the other by LDS DMA (global_load_lds: no VGPRs, and the compiler does not
// wait on it for reads of the other buffer -- a distinct __shared__ array), and the next tile's own
// per-pixel loads are in flight in registers; the one barrier per tile waits for both.  This hides the
// staging latency that one-tile blocks expose at every block start, amortises the table loads over the
// block's tiles and removes the grid's last partial wave of blocks.
struct TileWalk {
    uint32_t t, end, step;
    __device__ __forceinline__ TileWalk(uint32_t n_tiles) {
        const uint32_t per = (n_tiles + 7u) >> 3, x = blockIdx.x & 7u;
        const uint32_t start = min(x * per, n_tiles);
        end = min(start + per, n_tiles);
        step = gridDim.x >> 3;
        t = start + (blockIdx.x >> 3);
    }
    __device__ __forceinline__ bool valid(uint32_t u) const { return u < end; }
};

// One 16x16 tile's footprint of a same-size A = STD pass: (16 + 2R)^2 BGRA8 words, row-major, clamped to
// the texture, by LDS DMA into `buf` (each wave-instruction fills 64 consecutive words).
template <int STD>
struct FinalStd {
    static constexpr int RCH = 2 * (STD / 8);  // the taps' reach: |offset| <= 2 * A / 8 texels
    static constexpr int NX = 16 + 2 * RCH, NN = NX * NX, ROUNDS = (NN + 255) / 256;
};
template <int STD>
__device__ __forceinline__ void stage_final_dma(const CTex& U, uint32_t t, uint32_t tiles_x, uint32_t* buf) {
    using F = FinalStd<STD>;
    const uint32_t ty = t / tiles_x, tx = t - ty * tiles_x;
    const int32_t x0 = (int32_t)tx * 16 - F::RCH, y0 = (int32_t)ty * 16 - F::RCH;
    const int32_t wm = (int32_t)U.w - 1, hm = (int32_t)U.h - 1;
#pragma unroll
    for (int r = 0; r < F::ROUNDS; ++r) {
        const int32_t i = r * 256 + (int32_t)threadIdx.x;
        if (r * 256 + (int32_t)(threadIdx.x & ~63u) < F::NN) {  // wave-uniform: whole 64-word runs
            const int32_t ly = min(i, F::NN - 1) / F::NX, lx = min(i, F::NN - 1) - ly * F::NX;
            const uint32_t* g = U.px + (uint32_t)clampi(y0 + ly, 0, hm) * U.w + clampi(x0 + lx, 0, wm);
            __builtin_amdgcn_global_load_lds(g, buf + r * 256 + (threadIdx.x & ~63u), 4, 0, 0);
        }
    }
}
// Fused last stage (bloom_final_kernel) with the standard plan A = STD, persistent.
template <int STD>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7)))
bloom_final_pkernel(Tables tb, CTex col, CTex Y, CTex U0, TapPlan P, Tex out, uint32_t tiles_x, uint32_t n_tiles) {
    using F = FinalStd<STD>;
    static_assert(F::NN % 64 == 0, "whole 64-word DMA runs");
    __shared__ Lds L;
    __shared__ uint32_t B0[F::NN], B1[F::NN];
    TileWalk w(n_tiles);
    const int32_t lx = (int32_t)(threadIdx.x & 15u), ly = (int32_t)(threadIdx.x >> 4);
    auto pix = [&](uint32_t t, int32_t& x, int32_t& y) {
        const uint32_t ty = t / tiles_x;
        x = (int32_t)(t - ty * tiles_x) * 16 + lx;
        y = (int32_t)ty * 16 + ly;
    };
    auto fetch_px = [&](uint32_t t, uint32_t& yv, uint32_t& cv) {
        int32_t x, y;
        pix(t, x, y);
        const bool in = x < (int32_t)out.w && y < (int32_t)out.h;
        const uint32_t i = in ? (uint32_t)y * out.w + (uint32_t)x : 0;
        yv = Y.px[i];
        cv = col.px[i];
    };
    uint32_t yv = 0, cv = 0;
    if (w.valid(w.t)) {
        fetch_px(w.t, yv, cv);
        stage_final_dma<STD>(U0, w.t, tiles_x, B0);
    }
    load_tables(tb, L);
    // one tile from `cur` while the next streams into `nxt` (the loop is unrolled by two so that each
    // buffer stays a distinct array in the code)
    auto tile = [&](const uint32_t* cur, uint32_t* nxt) -> bool {
        if (!w.valid(w.t)) return false;  // block-uniform
        // cur's DMA (every wave's share) and this tile's pixel loads landed, nxt's last readers are done:
        // each wave drains its own vector-memory counter first (the compiler does not count the LDS
        // DMA's writes as LDS stores that the barrier must order), then the barrier
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const uint32_t t = w.t, tn = t + w.step;
        uint32_t yn = 0, cn = 0;
        if (w.valid(tn)) {
            fetch_px(tn, yn, cn);
            stage_final_dma<STD>(U0, tn, tiles_x, nxt);
        }
        int32_t x, y;
        pix(t, x, y);
        if (x < (int32_t)out.w && y < (int32_t)out.h) {
            const int32_t x0 = x - lx - F::RCH, y0 = y - ly - F::RCH;
            const PlanSrc<F::NX, true, STD> src{U0, cur, x0, y0, &P, &L, x, y};
            const F4 b3 = quant(L, up8(src, Taps(1u, 1u), 0.0f, 0.0f, 0u));
            const F4 z = quant(L, remix(dec(L, yv), b3));
            out.px[(uint32_t)y * out.w + (uint32_t)x] = enc(L, remix(dec(L, cv), z));
        }
        yv = yn;
        cv = cn;
        w.t = tn;
        return true;
    };
    while (tile(B0, B1) && tile(B1, B0)) {
    }
}

// The 2:1 form of an 8-tap pass: an up pass from a texture of n texels to 2n pixels along each axis
// (at 4096x2048 the full-size up pass from 2048x1024 and the one before it).  Its taps' texel
// coordinates are t = (x >> 1) + o + f with an integer o and a weight f in [0, 1) that depend only on
// the pixel's parity and the tap (the host proves it for every pixel: up2_plan), and o of an odd
// pixel is o of an even one or one more.  Where no tap is clamped and both texels of every tap lie
// inside the texture (the interior: every block but the outermost ring), the bilinear sample reads
// texels (x>>1) + o and + 1 with weights f, 1 - f -- the general sampler's own arithmetic, without its
// texcoord, floor and clamp work.  One lane computes a 2x2 pixel quad: per tap the four pixels' texels
// lie in a 3x3 (2x2 when both parities share o) neighbourhood of (x>>1, y>>1), read once for all four.

struct Up2Plan {
    int32_t ox[2][8], oy[2][8];      // [pixel parity][tap]: floor(t) - (x >> 1)
    float fx[2][8], fy[2][8];        // t - floor(t)
    int32_t x_lo, x_hi, y_lo, y_hi;  // the interior's output pixels (inclusive; empty when lo > hi)
    uint32_t valid;
};

// bilinear of texels (t00, t10, t01, t11) with weights (fa, fb): sample()'s operations in its order
__device__ __forceinline__ F4 lerp2(const float4& t00, const float4& t10, const float4& t01, const float4& t11, float fa,
                                    float fb) {
    const float ia = 1.0f - fa, ib = 1.0f - fb;
    F4 q;
    q.r = (t00.x * ia + t10.x * fa) * ib + (t01.x * ia + t11.x * fa) * fb;
    q.g = (t00.y * ia + t10.y * fa) * ib + (t01.y * ia + t11.y * fa) * fb;
    q.b = (t00.z * ia + t10.z * fa) * ib + (t01.z * ia + t11.z * fa) * fb;
    q.a = (t00.w * ia + t10.w * fa) * ib + (t01.w * ia + t11.w * fa) * fb;
    return q;
}
// One tap for the quad: DX / DY = o(odd) - o(even) along x / y; T = the (2 + DY) x (2 + DX) texels from
// (x>>1) + o(even), row stride FP.  s[b][a]: the pixel of y parity b, x parity a.
template <int FP, int DX, int DY>
__device__ __forceinline__ void quad_tap(const float4* T, const Up2Plan& P, int i, F4 (&s)[2][2]) {
    float4 t[2 + DY][2 + DX];
#pragma unroll
    for (int r = 0; r < 2 + DY; ++r)
#pragma unroll
        for (int c = 0; c < 2 + DX; ++c) t[r][c] = T[r * FP + c];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const int c = a ? DX : 0, r = b ? DY : 0;
            acc(s[b][a], lerp2(t[r][c], t[r][c + 1], t[r + 1][c], t[r + 1][c + 1], P.fx[a][i], P.fy[b][i]), i);
        }
}

// ---- compile-time plans of the standard chain ---------------------------------------------------
// On power-of-two frames at levels 3 (the reference's chain: src/state.rs:125) every 8-tap pass has the
// same plan whatever the size, because each tap's texel offset scales with the texture: tap (mx, my)'s
// coordinate along an axis is  x + A*m/8  (same-size passes: Y, A = 12; the final pass, A = 48) or
// (x >> 1) + (A*m -+ 2)/8 for even / odd pixels (2:1 up passes: the half-size one A = 3, the full-size
// one A = 12), in eighths of a texel.  A kernel instantiated for such an A reads every tap at constant
// LDS offsets with constant weights: no plan loads, no per-tap branches, and the exact forms below.  The
// host takes it only when the plan it proves for the launch (tap_plan / up2_plan) equals this one
// entry for entry (std_tap_plan / std_up2_plan); otherwise the runtime-plan kernels run.
// a lerp t0 (1 - f) + t1 f with f = F/8 known: f = 0 returns t0 (t0 * 1 + t1 * 0); when one weight is a
// power of two its product is exact (texels and their lerps are 0 or far from the subnormals), so the
// sum is one fma on the other product -- RN(RN(t0 g) + t1 f) == fma(t1, f, RN(t0 g)) -- the same bits
template <int F>
__device__ __forceinline__ float clerp(float t0, float t1) {
    constexpr float f = (float)F / 8.0f, g = 1.0f - f;
    if constexpr (F == 0) return t0;
    else if constexpr (F == 1 || F == 2 || F == 4) return __builtin_fmaf(t1, f, t0 * g);
    else if constexpr (F == 6 || F == 7) return __builtin_fmaf(t0, g, t1 * f);
    else return t0 * g + t1 * f;
}
template <int FA, int FB>
__device__ __forceinline__ F4 clerp2(const float4& t00, const float4& t10, const float4& t01, const float4& t11) {
    F4 q;
    q.r = clerp<FB>(clerp<FA>(t00.x, t10.x), clerp<FA>(t01.x, t11.x));
    q.g = clerp<FB>(clerp<FA>(t00.y, t10.y), clerp<FA>(t01.y, t11.y));
    q.b = clerp<FB>(clerp<FA>(t00.z, t10.z), clerp<FA>(t01.z, t11.z));
    q.a = clerp<FB>(clerp<FA>(t00.w, t10.w), clerp<FA>(t01.w, t11.w));
    return q;
}
// tap I of a 2:1 up pass with the standard plan A, for the quad at `base` (the even pixels' texel)
template <int FP, int A, int I>
__device__ __forceinline__ void quad_tap_std(const float4* base, F4 (&s)[2][2]) {
    constexpr int vx0 = A * tap_m(0, I) - 2, vx1 = A * tap_m(0, I) + 2;
    constexpr int vy0 = A * tap_m(1, I) - 2, vy1 = A * tap_m(1, I) + 2;
    constexpr int DX = fdiv8(vx1) - fdiv8(vx0), DY = fdiv8(vy1) - fdiv8(vy0);
    static_assert((DX == 0 || DX == 1) && (DY == 0 || DY == 1), "the quad's texels span 2 or 3 per axis");
    const float4* T = base + fdiv8(vy0) * FP + fdiv8(vx0);
    float4 t[2 + DY][2 + DX];
#pragma unroll
    for (int r = 0; r < 2 + DY; ++r)
#pragma unroll
        for (int c = 0; c < 2 + DX; ++c) t[r][c] = T[r * FP + c];
    acc(s[0][0], clerp2<fmod8(vx0), fmod8(vy0)>(t[0][0], t[0][1], t[1][0], t[1][1]), I);
    acc(s[0][1], clerp2<fmod8(vx1), fmod8(vy0)>(t[0][DX], t[0][DX + 1], t[1][DX], t[1][DX + 1]), I);
    acc(s[1][0], clerp2<fmod8(vx0), fmod8(vy1)>(t[DY][0], t[DY][1], t[DY + 1][0], t[DY + 1][1]), I);
    acc(s[1][1], clerp2<fmod8(vx1), fmod8(vy1)>(t[DY][DX], t[DY][DX + 1], t[DY + 1][DX], t[DY + 1][DX + 1]), I);
}
template <int FP, int A, int... I>
__device__ __forceinline__ void quad_taps_std(const float4* base, F4 (&s)[2][2], std::integer_sequence<int, I...>) {
    // one tap at a time: the sched barrier keeps the next tap's reads from being hoisted over this one's
    // arithmetic, pin() keeps this tap's arithmetic from sinking below the next
    ((quad_tap_std<FP, A, I>(base, s), pin(s), __builtin_amdgcn_sched_barrier(0)), ...);
}

// A 2:1 up pass (kawase_upsample.wgsl): 32x32 pixels per 256-thread block, one 2x2 quad per lane; the
// outermost blocks (and footprints over FP) take the general sampler per pixel.  STD: 0 = the runtime
// plan P, else the standard plan A = STD (P still gives the interior).
constexpr int FP_UPQ = 28;  // footprint of 16 texels + the taps' reach (24 at 4096x2048)
// row stride in float4, a multiple of 16: here lane l reads texel column (l & 15) + c (a 2:1 pass reads
// one texel per output quad), 16 consecutive slots per quad row, and the lane groups take two quad rows
// (see FS_YQ): with 28 the second row overlapped the first's slots (bank conflicts 0.42 of LDS-active
// cycles), with 32 it lands on the same slots of the next 64 banks (0.01)
constexpr int FS_UPQ = 32;
template <int STD>
__global__ void BLOOM_BOUNDS up2_kernel(Tables tb, CTex a, uint32_t rx, uint32_t ry, uint32_t point, Up2Plan P,
                                        Tex out) {
    __shared__ Lds L;
    __shared__ float4 tile[FP_UPQ * FS_UPQ];
    const uint32_t bx = xcd_block().x * 32u, by = xcd_block().y * 32u;
    const uint32_t x = bx + 2u * (threadIdx.x & 15u), y = by + 2u * (threadIdx.x >> 4);  // the quad's corner
    const crm::Rcp Rw = crm::rcp_refined((float)out.w), Rh = crm::rcp_refined((float)out.h);
    const Taps k(rx, ry);
    const Span sx = tap_span(bx, min(bx + 31u, out.w - 1u), Rw, k.du_min(), k.du_max(), a.w);
    const Span sy = tap_span(by, min(by + 31u, out.h - 1u), Rh, k.dv_min(), k.dv_max(), a.h);
    const bool staged = sx.n <= FP_UPQ && sy.n <= FP_UPQ;  // block-uniform
    if (staged) {
        // every load of this thread first, then the decodes (as with_source)
        constexpr int R = (FP_UPQ * FP_UPQ + 255) / 256;
        uint32_t raw[R];
        const int32_t n = sx.n * sy.n;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int32_t i = (int32_t)threadIdx.x + r * 256;
            if (i < n) {
                const int32_t ly = i / sx.n, lx = i - ly * sx.n;
                raw[r] = a.px[(uint32_t)(sy.lo + ly) * a.w + (sx.lo + lx)];
            }
        }
        load_tables(tb, L);  // after the footprint's loads are issued: both round trips overlap
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int32_t i = (int32_t)threadIdx.x + r * 256;
            if (i < n) {
                const int32_t ly = i / sx.n, lx = i - ly * sx.n;
                const F4 d = dec(L, raw[r]);
                tile[ly * FS_UPQ + lx] = make_float4(d.r, d.g, d.b, d.a);
            }
        }
        __syncthreads();
    } else {
        load_tables(tb, L);
    }
    if (x >= out.w || y >= out.h) return;  // out.w, out.h are even (2n): the whole quad is outside
    const bool inner = staged && (int32_t)bx >= P.x_lo && (int32_t)bx + 31 <= P.x_hi && (int32_t)by >= P.y_lo &&
                       (int32_t)by + 31 <= P.y_hi;  // block-uniform
    if (!inner) {
        // the general sampler per pixel (rolled: four unrolled 8-tap samples need 120 VGPRs)
#pragma unroll 1
        for (int j = 0; j < 4; ++j) {
            const uint32_t px = x + (j & 1), py = y + (j >> 1);
            const float u = texcoord(px, Rw), v = texcoord(py, Rh);
            const F4 r = staged ? up8(TileSrc<FS_UPQ>{a, tile, sx.lo, sy.lo}, k, u, v, point)
                                : up8(GlobalSrc{a, &L}, k, u, v, point);
            out.px[(uint32_t)py * out.w + px] = enc(L, r);
        }
        return;
    }
    F4 s[2][2];
    const int32_t base = ((int32_t)(y >> 1) - sy.lo) * FS_UPQ + ((int32_t)(x >> 1) - sx.lo);
    if constexpr (STD != 0) {
        quad_taps_std<FS_UPQ, STD>(tile + base, s, std::make_integer_sequence<int, 8>{});
    } else {
        // rolled (the plan read by scalar loads; unrolled, the taps' LDS reads are hoisted together)
#pragma unroll 1
        for (int i = 0; i < 8; i++) {
            const float4* T = tile + (base + P.oy[0][i] * FS_UPQ + P.ox[0][i]);
            const uint32_t d = (uint32_t)(P.ox[1][i] - P.ox[0][i]) | (uint32_t)(P.oy[1][i] - P.oy[0][i]) << 1;
            switch (d) {  // wave-uniform
                case 0: quad_tap<FS_UPQ, 0, 0>(T, P, i, s); break;
                case 1: quad_tap<FS_UPQ, 1, 0>(T, P, i, s); break;
                case 2: quad_tap<FS_UPQ, 0, 1>(T, P, i, s); break;
                default: quad_tap<FS_UPQ, 1, 1>(T, P, i, s); break;
            }
        }
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        uint2 w;
        w.x = enc(L, div12(s[b][0]));
        w.y = enc(L, div12(s[b][1]));
        *reinterpret_cast<uint2*>(out.px + (uint32_t)(y + b) * out.w + x) = w;  // x even: 8-byte aligned
    }
}

}  // namespace bloom
}  // namespace bh

using namespace bh::bloom;

namespace {
dim3 grid_for(uint32_t w, uint32_t h) { return dim3((w + 15u) / 16u, (h + 15u) / 16u); }
}  // namespace

// Host side of the point-tap proof: the kernels' texcoord / tap / sample_coord arithmetic in IEEE f32
// (identical on the host: no contraction in this file, and div_core == IEEE division in its domain).
namespace {
float h_sample_coord(float u, uint32_t n) {
    const float t = u * (float)n - 0.5f;
    return fminf(fmaxf(t, -1.0f), (float)n);
}
bool axis_point(uint32_t on, uint32_t tn, float d) {
    for (uint32_t x = 0; x < on; ++x) {
        const float t = h_sample_coord(((float)x + 0.5f) / (float)on + d, tn);
        if (t != floorf(t)) return false;
    }
    return true;
}
}  // namespace

// One axis of tap i (offset d in texcoord units) over an on-pixel pass of an tn-texel texture: the
// integer offset o and half flag f with u*tn - 0.5 == x + o + f/2 exactly for every x, else false.
bool axis_plan(uint32_t on, uint32_t tn, float d, int32_t* o, bool* half) {
    const float t0 = ((0.5f / (float)on) + d) * (float)tn - 0.5f;
    const float f0 = floorf(t0);
    if (!(t0 - f0 == 0.0f || t0 - f0 == 0.5f) || !(fabsf(f0) < 4096.0f)) return false;
    *o = (int32_t)f0;
    *half = t0 != f0;
    const float fr = t0 - f0;
    for (uint32_t x = 0; x < on; ++x) {
        const float t = (((float)x + 0.5f) / (float)on + d) * (float)tn - 0.5f;
        if (t != (float)((int32_t)x + *o) + fr) return false;
    }
    return true;
}
struct PlanKey { uint32_t ow, oh, tw, th, rx, ry; };
// The TapPlan of an 8-tap pass (see TapPlan), cached per shape (a few per bloom chain).
TapPlan tap_plan(uint32_t ow, uint32_t oh, uint32_t tw, uint32_t th, uint32_t rx, uint32_t ry) {
    static thread_local PlanKey keys[16];
    static thread_local TapPlan plans[16];
    static thread_local uint32_t n = 0, next = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (keys[i].ow == ow && keys[i].oh == oh && keys[i].tw == tw && keys[i].th == th && keys[i].rx == rx &&
            keys[i].ry == ry)
            return plans[i];
    TapPlan P{};
    P.valid = 1u;
    P.lo_x = P.lo_y = 1 << 20;
    P.hi_x = P.hi_y = -(1 << 20);
    const float hx = 0.5f / (float)rx, hy = 0.5f / (float)ry;
    for (int i = 0; i < 8 && P.valid; ++i) {
        const float du = (hx * (float)((int)((0x12343210u >> (4 * i)) & 15u) - 2)) * 3.0f;
        const float dv = (hy * (float)((int)((0x10123432u >> (4 * i)) & 15u) - 2)) * 3.0f;
        bool fx, fy;
        if (!axis_plan(ow, tw, du, &P.ox[i], &fx) || !axis_plan(oh, th, dv, &P.oy[i], &fy)) {
            P.valid = 0u;
            break;
        }
        P.hx |= (uint32_t)fx << i;
        P.hy |= (uint32_t)fy << i;
        P.lo_x = std::min(P.lo_x, P.ox[i]); P.hi_x = std::max(P.hi_x, P.ox[i] + (int32_t)fx);
        P.lo_y = std::min(P.lo_y, P.oy[i]); P.hi_y = std::max(P.hi_y, P.oy[i] + (int32_t)fy);
    }
    if (!P.valid) P = TapPlan{};
    keys[next] = {ow, oh, tw, th, rx, ry};
    plans[next] = P;
    next = (next + 1u) % 16u;
    n = n < 16u ? n + 1u : 16u;
    return P;
}

// One axis of tap i (offset d in texcoord units) of a 2:1 pass (on == 2 tn): per pixel parity p the
// integer o[p] and weight f[p] with floor(t) == (x >> 1) + o[p] and t - floor(t) == f[p] for every x,
// t = u*tn - 0.5 the sampler's unclamped coordinate; [lo, hi] = the pixels whose two texels floor(t),
// floor(t) + 1 both lie in [0, tn) (there the sampler's clamps change nothing).  False if not so.
bool axis_plan2(uint32_t on, uint32_t tn, float d, int32_t o[2], float f[2], int32_t* lo, int32_t* hi) {
    if (on != 2u * tn || tn < 2u) return false;
    bool seen[2] = {false, false};
    int32_t ilo = INT_MAX, ihi = -1, count = 0;
    for (uint32_t x = 0; x < on; ++x) {
        const float t = (((float)x + 0.5f) / (float)on + d) * (float)tn - 0.5f;
        const float fl = floorf(t);
        if (!(fabsf(fl) < 16777216.0f)) return false;
        const uint32_t p = x & 1u;
        const int32_t oo = (int32_t)fl - (int32_t)(x >> 1);
        const float ff = t - fl;
        if (!seen[p]) {
            o[p] = oo;
            f[p] = ff;
            seen[p] = true;
        } else if (oo != o[p] || std::memcmp(&ff, &f[p], sizeof ff) != 0) {
            return false;
        }
        if (fl >= 0.0f && fl + 1.0f <= (float)tn - 1.0f) {
            ilo = std::min(ilo, (int32_t)x);
            ihi = std::max(ihi, (int32_t)x);
            ++count;
        }
    }
    if (count != 0 && count != ihi - ilo + 1) return false;  // t is monotone: an interval
    *lo = count ? ilo : 0;
    *hi = count ? ihi : -1;
    return true;
}
// The Up2Plan of an up pass (see Up2Plan), cached per shape; valid == 0 when the pass is not 2:1 or a
// tap's offset or weight varies within a parity class.
Up2Plan up2_plan(uint32_t ow, uint32_t oh, uint32_t tw, uint32_t th, uint32_t rx, uint32_t ry) {
    static thread_local PlanKey keys[16];
    static thread_local Up2Plan plans[16];
    static thread_local uint32_t n = 0, next = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (keys[i].ow == ow && keys[i].oh == oh && keys[i].tw == tw && keys[i].th == th && keys[i].rx == rx &&
            keys[i].ry == ry)
            return plans[i];
    Up2Plan P{};
    P.valid = 1u;
    P.x_lo = P.y_lo = 0;
    P.x_hi = (int32_t)ow - 1;
    P.y_hi = (int32_t)oh - 1;
    const float hx = 0.5f / (float)rx, hy = 0.5f / (float)ry;
    for (int i = 0; i < 8; ++i) {
        const float du = (hx * (float)((int)((0x12343210u >> (4 * i)) & 15u) - 2)) * 3.0f;
        const float dv = (hy * (float)((int)((0x10123432u >> (4 * i)) & 15u) - 2)) * 3.0f;
        int32_t ox[2], oy[2], xl, xh, yl, yh;
        float fx[2], fy[2];
        if (!axis_plan2(ow, tw, du, ox, fx, &xl, &xh) || !axis_plan2(oh, th, dv, oy, fy, &yl, &yh)) {
            P.valid = 0u;
            break;
        }
        for (int p = 0; p < 2; ++p) {
            P.ox[p][i] = ox[p]; P.fx[p][i] = fx[p];
            P.oy[p][i] = oy[p]; P.fy[p][i] = fy[p];
        }
        if (ox[1] - ox[0] < 0 || ox[1] - ox[0] > 1 || oy[1] - oy[0] < 0 || oy[1] - oy[0] > 1) {  // the quad's 3x3
            P.valid = 0u;
            break;
        }
        P.x_lo = std::max(P.x_lo, xl); P.x_hi = std::min(P.x_hi, xh);
        P.y_lo = std::max(P.y_lo, yl); P.y_hi = std::min(P.y_hi, yh);
    }
    if (!P.valid) P = Up2Plan{};
    keys[next] = {ow, oh, tw, th, rx, ry};
    plans[next] = P;
    next = (next + 1u) % 16u;
    n = n < 16u ? n + 1u : 16u;
    return P;
}

// Grid of a persistent bloom kernel: `per_cu` resident blocks on every CU of the current device, a
// multiple of 8 (TileWalk splits the tiles into 8 runs).
uint32_t persistent_grid(uint32_t per_cu) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
        cus = 256;
    return std::max(8u, ((uint32_t)cus * per_cu) & ~7u);
}

// The standard plan (see quad_tap_std) a runtime plan equals, or 0: A = 12 or 3 for a 2:1 up pass, A =
// 12 or 48 for a same-size TapPlan pass.  BH_BLOOM_NO_STD (A/B) disables them.
static const bool g_no_std = std::getenv("BH_BLOOM_NO_STD") != nullptr;
int std_up2_plan(const Up2Plan& P) {
    if (!P.valid || g_no_std) return 0;
    for (int A : {12, 3}) {
        bool eq = true;
        for (int i = 0; i < 8 && eq; ++i)
            for (int p = 0; p < 2 && eq; ++p) {
                const int vx = A * tap_m(0, i) + (p ? 2 : -2), vy = A * tap_m(1, i) + (p ? 2 : -2);
                eq = P.ox[p][i] == fdiv8(vx) && P.oy[p][i] == fdiv8(vy) && P.fx[p][i] == (float)fmod8(vx) / 8.0f &&
                     P.fy[p][i] == (float)fmod8(vy) / 8.0f;
            }
        if (eq) return A;
    }
    return 0;
}
int std_tap_plan(const TapPlan& P) {
    if (!P.valid || g_no_std) return 0;
    for (int A : {12, 48}) {
        bool eq = true;
        for (int i = 0; i < 8 && eq; ++i) {
            const int vx = A * tap_m(0, i), vy = A * tap_m(1, i);
            eq = (fmod8(vx) == 0 || fmod8(vx) == 4) && (fmod8(vy) == 0 || fmod8(vy) == 4) && P.ox[i] == fdiv8(vx) &&
                 P.oy[i] == fdiv8(vy) && ((P.hx >> i) & 1u) == (fmod8(vx) == 4 ? 1u : 0u) &&
                 ((P.hy >> i) & 1u) == (fmod8(vy) == 4 ? 1u : 0u);
        }
        if (eq) return A;
    }
    return 0;
}

// ---- host-side bound checks of the kernels' index arithmetic ------------------------------------
// Round 4's memory-access fault ("Bound checks") was a fix-up launch with a count read
// from a freed plan record.  Every form a launcher can take stages a block's input footprint in an LDS
// tile and reads it at offsets that a plan (or the kernel's own sampler arithmetic) gives; these checks
// replay that arithmetic on the host, in the kernels' own f32 operations, per block and per tap along
// each axis (every footprint here is separable), and require every staged extent to fit its tile, every
// tile read to fall inside the staged extent, and every plan index and list entry to fall inside its
// texture.  A separable or same-size plan that fails is never used (the pass takes the general form:
// bh_bloom_sep_verify / bh_bloom_same_verify, called where the host builds the plans), and in the dry
// mode of bh_bloom_check every launch of a chain runs its form's check instead of launching (the CPU
// test over frame sizes and levels, tests/test_bloom_bounds.py).
namespace {
struct DryRun {
    uint64_t launches = 0, checks = 0;
    std::string fail;
    std::string plan;  // one line per launch: its form, output size, input size, resolution uniform
};
thread_local DryRun* g_dry = nullptr;
// Test hook (tests/test_bloom_bounds.py): the checks treat every tile as this many entries smaller, so a
// footprint that fills its tile exactly must be reported -- the checks' own negative test.  0 in use.
const int g_check_slack = [] {
    const char* e = std::getenv("BH_BLOOM_CHECK_SLACK");
    return e ? std::atoi(e) : 0;
}();
thread_local std::string* g_why = nullptr;  // where a failing check writes its message (first one kept)

bool chk(bool ok, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
bool chk(bool ok, const char* fmt, ...) {
    if (g_dry) ++g_dry->checks;
    if (ok) return true;
    std::string* w = g_dry ? &g_dry->fail : g_why;
    if (w && w->empty()) {
        char buf[256];
        va_list ap;
        va_start(ap, fmt);
        std::vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        *w = buf;
    }
    return false;
}
// the dry run's launch list (bh_bloom_check): "form ow oh tw th rx ry"
void note_launch(const char* form, uint32_t ow, uint32_t oh, uint32_t tw, uint32_t th, uint32_t rx, uint32_t ry) {
    if (!g_dry) return;
    ++g_dry->launches;
    char buf[128];
    std::snprintf(buf, sizeof buf, "%s %u %u %u %u %u %u\n", form, ow, oh, tw, th, rx, ry);
    g_dry->plan += buf;
}
float h_texcoord(uint32_t i, uint32_t n) { return ((float)i + 0.5f) / (float)n; }
// Taps::du / dv on the host: (hx * m) * 3 with hx = 0.5 / res
float h_tap(uint32_t res, int axis, int i) { return ((0.5f / (float)res) * (float)tap_m(axis, i)) * 3.0f; }
float h_tap_min(uint32_t res, int axis) { return h_tap(res, axis, axis ? 6 : 0); }
float h_tap_max(uint32_t res, int axis) { return h_tap(res, axis, axis ? 2 : 4); }
int32_t h_floor(float t) { return (int32_t)floorf(t); }

// One axis of up_sep_kernel (B = 16) / up_sepq_kernel (B = 32): the footprint the kernel derives from the
// sampler arithmetic of its first and last column, c = hi - lo + 2 entries (floor .. floor + 1), which the
// kernel cuts to FP -- the cut must never happen -- and for every tap and column of the block the plan's
// floor f with both of its texels f - lo, f + 1 - lo inside those c entries.  e: the axis's [8][on] entries.
// off: the block grid's origin offset (blocks start at B k - off; the quad kernel's org), own: the block's own
// columns must lie in its footprint too (the FIX epilogue reads them from the tile).
bool sep_axis_ok(const SepEntry* e, uint32_t on, uint32_t tn, uint32_t res, int axis, uint32_t B, int FP, uint32_t off = 0,
                 bool own = false) {
    const float dmin = h_tap_min(res, axis), dmax = h_tap_max(res, axis);
    if (!chk(off < B && off % 2u == 0u, "block grid origin %u for %u-pixel blocks", off, B)) return false;
    for (int64_t bs = -(int64_t)off; bs < (int64_t)on; bs += B) {
        const uint32_t b = (uint32_t)std::max<int64_t>(bs, 0);
        const uint32_t l = (uint32_t)std::min<int64_t>(bs + B - 1, (int64_t)on - 1);
        const int32_t lo = h_floor(h_sample_coord(h_texcoord(b, on) + dmin, tn));
        const int32_t hi = h_floor(h_sample_coord(h_texcoord(l, on) + dmax, tn));
        const int32_t c = hi - lo + 2;
        if (!chk(c >= 2 && c <= FP - g_check_slack, "separable %s footprint of block %u: %d entries, tile side %d", axis ? "row" : "column",
                 b, c, FP))
            return false;
        if (own && !chk((int32_t)b - lo >= 0 && (int32_t)l - lo <= c - 1,
                        "in-block fix: %s block %u..%u outside its footprint %d + %d", axis ? "row" : "column", b, l, lo, c))
            return false;
        for (int i = 0; i < 8; ++i)
            for (uint32_t x = b; x <= l; ++x) {
                const SepEntry& s = e[(size_t)i * on + x];
                if (!chk(s.f >= -1 && s.f <= (int32_t)tn, "separable plan floor %d outside [-1, %u] (tap %d, %s %u)", s.f,
                         tn, i, axis ? "row" : "column", x) ||
                    !chk(s.f - lo >= 0 && s.f + 1 - lo <= c - 1,
                         "separable tap %d of %s %u reads entries %d..%d of a %d-entry footprint", i, axis ? "row" : "column",
                         x, s.f - lo, s.f + 1 - lo, c) ||
                    !chk(s.fa >= 0.0f && s.fa <= 1.0f && s.ia == 1.0f - s.fa, "separable plan weight %g at %s %u", (double)s.fa,
                         axis ? "row" : "column", x))
                    return false;
            }
    }
    return true;
}
// A tile of FP rows at stride FS, with a row-pair shift of (ly + p) >> 1 entries when shift = p + 1 (the quad
// tiles: p = 0; bloom_yq_kernel: p up to 1): its largest entry for rows and columns below FP must stay below
// the declared size.
bool tile_ok(int FP, int FS, int shift, int size) {
    const int last = (FP - 1) * FS + (shift ? (FP - 1 + shift - 1) >> 1 : 0) + (FP - 1);
    return chk(FS >= FP && last < size, "tile FP %d stride %d: last entry %d of %d", FP, FS, last, size);
}

// One axis of with_source's (and up2_kernel's outer blocks') fallback: the kernel's tap_span over a block of
// B pixels, and, when it fits FP, every tap's two clamped texels inside it.
bool span_axis_ok(uint32_t on, uint32_t tn, uint32_t res, int axis, uint32_t B, int FP) {
    const float dmin = h_tap_min(res, axis), dmax = h_tap_max(res, axis);
    const int32_t hm = (int32_t)tn - 1;
    auto clampi_h = [&](int32_t v) { return std::min(std::max(v, 0), hm); };
    for (uint32_t b = 0; b < on; b += B) {
        const uint32_t l = std::min(b + B - 1u, on - 1u);
        const int32_t lo = clampi_h(h_floor(h_sample_coord(h_texcoord(b, on) + dmin, tn)));
        const int32_t hi = clampi_h(h_floor(h_sample_coord(h_texcoord(l, on) + dmax, tn)) + 1);
        const int32_t n = hi - lo + 1;
        if (n > FP) continue;  // block-uniform: this block reads global memory through clamped indices
        if (!chk(n <= FP - g_check_slack, "staged span of %s block %u: %d texels, tile side %d", axis ? "row" : "column",
                 b, n, FP))
            return false;
        for (int i = 0; i < 8; ++i)
            for (uint32_t x = b; x <= l; ++x) {
                const int32_t f = h_floor(h_sample_coord(h_texcoord(x, on) + h_tap(res, axis, i), tn));
                const int32_t x0 = clampi_h(f), x1 = clampi_h(f + 1);
                if (!chk(x0 >= lo && x1 <= hi, "staged tap %d of %s %u reads texels %d..%d of span %d..%d", i,
                         axis ? "row" : "column", x, x0, x1, lo, hi))
                    return false;
            }
    }
    return true;
}

// One axis of a TapPlan form over blocks of B pixels and a tile of side FP: the kernel takes the form when
// hi - lo + B <= FP (launch-uniform), and then a pixel p of a block reads entries p - b + (o_i - lo) and
// + half_i; otherwise the span fallback.
bool tapplan_axis_ok(const TapPlan& P, uint32_t on, uint32_t tn, uint32_t res, int axis, uint32_t B, int FP) {
    const int32_t lo = axis ? P.lo_y : P.lo_x, hi = axis ? P.hi_y : P.hi_x;
    if (!P.valid || hi - lo + (int32_t)B > FP) return span_axis_ok(on, tn, res, axis, B, FP);
    if (!chk(hi - lo + (int32_t)B <= FP - g_check_slack, "tap plan footprint %d of a %d tile", hi - lo + (int32_t)B, FP))
        return false;
    for (int i = 0; i < 8; ++i) {
        const int32_t o = axis ? P.oy[i] : P.ox[i];
        const int32_t h = (int32_t)(((axis ? P.hy : P.hx) >> i) & 1u);
        if (!chk(o - lo >= 0 && (int32_t)B - 1 + o + h - lo <= hi - lo + (int32_t)B - 1,
                 "tap plan tap %d offset %d (+%d) outside the footprint %d..%d", i, o, h, lo, hi))
            return false;
    }
    return true;
}

// One axis of up2_kernel: blocks of 32 pixels staged when the span fits FP_UPQ; inside P's interior the quad
// reads texels (x >> 1) + o[0] .. (x >> 1) + o[1] + 1 of every tap, which must lie in the span.
bool up2_axis_ok(const Up2Plan& P, uint32_t on, uint32_t tn, uint32_t res, int axis, int FP) {
    if (!span_axis_ok(on, tn, res, axis, 32u, FP)) return false;
    const float dmin = h_tap_min(res, axis), dmax = h_tap_max(res, axis);
    const int32_t hm = (int32_t)tn - 1;
    const int32_t ilo = axis ? P.y_lo : P.x_lo, ihi = axis ? P.y_hi : P.x_hi;
    for (uint32_t b = 0; b < on; b += 32u) {
        const uint32_t l = std::min(b + 31u, on - 1u);
        const int32_t lo = std::min(std::max(h_floor(h_sample_coord(h_texcoord(b, on) + dmin, tn)), 0), hm);
        const int32_t hi = std::min(std::max(h_floor(h_sample_coord(h_texcoord(l, on) + dmax, tn)) + 1, 0), hm);
        if (hi - lo + 1 > FP || (int32_t)b < ilo || (int32_t)b + 31 > ihi) continue;  // not an inner block
        for (int i = 0; i < 8; ++i) {
            const int32_t o0 = axis ? P.oy[0][i] : P.ox[0][i], o1 = axis ? P.oy[1][i] : P.ox[1][i];
            for (uint32_t x = b; x <= l; x += 2u) {
                const int32_t first = (int32_t)(x >> 1) + o0, last = (int32_t)(x >> 1) + o1 + 1;
                if (!chk(first >= lo && last <= hi && first >= 0 && last <= hm,
                         "2:1 quad tap %d of %s %u reads texels %d..%d of span %d..%d", i, axis ? "row" : "column", x,
                         first, last, lo, hi))
                    return false;
            }
        }
    }
    return true;
}

// The same-size plan (bh_bloom_same_plan) and its list of inexact columns, then rows: every texel index
// inside the frame, weights in [0, 1], and the list exactly the columns / rows of nonzero weight, ascending
// (the fused epilogues skip those pixels and fixup_kernel recomputes them: a missing entry leaves a pixel
// unwritten, an extra one writes it twice with the same value).
bool same_ok(uint32_t w, uint32_t h, const uint32_t* plan, const uint32_t* list, uint32_t nc, uint32_t nr,
             bool with_list = true) {
    if (!chk(nc <= w && nr <= h, "same-size plan: %u inexact columns of %u, %u rows of %u", nc, w, nr, h)) return false;
    for (int axis = 0; axis < 2; ++axis) {
        const uint32_t n = axis ? h : w, base = axis ? w : 0u, cnt = axis ? nr : nc;
        const uint32_t* L = with_list ? list + (axis ? nc : 0u) : nullptr;
        uint32_t k = 0;
        for (uint32_t x = 0; x < n; ++x) {
            const uint32_t e = plan[2u * (base + x)];
            float wgt;
            std::memcpy(&wgt, &plan[2u * (base + x) + 1u], 4);
            const uint32_t x0 = e & 0xFFFFu, x1 = e >> 16;
            if (!chk(x0 < n && x1 < n && wgt >= 0.0f && wgt <= 1.0f, "same-size plan %s %u: texels %u, %u, weight %g of %u",
                     axis ? "row" : "column", x, x0, x1, (double)wgt, n) ||
                !chk(wgt != 0.0f || x0 == x, "same-size plan: exact %s %u samples texel %u", axis ? "row" : "column", x, x0))
                return false;
            if (wgt != 0.0f && with_list) {
                if (!chk(k < cnt && L[k] == x, "same-size list: %s %u missing", axis ? "row" : "column", x)) return false;
                ++k;
            }
        }
        if (with_list && !chk(k == cnt, "same-size list: %u %s entries for %u inexact", cnt, axis ? "row" : "column", k)) return false;
    }
    return true;
}
// Whether inexact column (row) x of an n-pixel axis samples a texel outside its 32-pixel block of a grid at
// origin off: such a column's pixels are the fix-up pass's, the others up_sepq_kernel's in-block fix (FIX).
// reach2 (the final epilogue's fix): also when a sampled texel is itself inexact and samples outside the block.
bool same_crosses(const uint32_t* plan, uint32_t base, uint32_t x, uint32_t off, bool reach2 = false) {
    const uint32_t e = plan[2u * (base + x)], wbits = plan[2u * (base + x) + 1u];
    if (wbits == 0u) return false;  // exact: its own texel (same_ok)
    const uint32_t blk = (x + off) / 32u;
    const uint32_t t[2] = {e & 0xFFFFu, e >> 16};  // both of nonzero weight (0 < w < 1)
    for (uint32_t u : t) {
        if ((u + off) / 32u != blk) return true;
        if (reach2 && plan[2u * (base + u) + 1u] != 0u) {
            const uint32_t eu = plan[2u * (base + u)];
            if (((eu & 0xFFFFu) + off) / 32u != blk || ((eu >> 16) + off) / 32u != blk) return true;
        }
    }
    return false;
}
// The residual list at origin org: the crossing columns, then rows, ascending -- exactly what it must hold
bool residual_ok(uint32_t w, uint32_t h, const uint32_t* plan, const uint32_t* list, uint32_t nc, uint32_t nr, uint32_t org,
                 bool reach2) {
    if (!chk(nc <= w && nr <= h && (org & 0xFFFFu) < 32u && (org >> 16) < 32u && org % 2u == 0u && (org >> 16) % 2u == 0u,
             "residual list: %u columns of %u, %u rows of %u, origin %u,%u", nc, w, nr, h, org & 0xFFFFu, org >> 16))
        return false;
    for (int axis = 0; axis < 2; ++axis) {
        const uint32_t n = axis ? h : w, base = axis ? w : 0u, cnt = axis ? nr : nc, off = axis ? org >> 16 : org & 0xFFFFu;
        const uint32_t* L = list + (axis ? nc : 0u);
        uint32_t k = 0;
        for (uint32_t x = 0; x < n; ++x)
            if (same_crosses(plan, base, x, off, reach2)) {
                if (!chk(k < cnt && L[k] == x, "residual list: crossing %s %u missing", axis ? "row" : "column", x)) return false;
                ++k;
            }
        if (!chk(k == cnt, "residual list: %u %s entries for %u crossing", cnt, axis ? "row" : "column", k)) return false;
    }
    return true;
}
// The fix-up records of a list (bh_bloom_fixup_records): entry k's column (row) and the plan entries of it and
// of its clamped neighbours, exactly as the kernel would read them from the plan.
bool records_ok(uint32_t w, uint32_t h, const uint32_t* plan, const uint32_t* list, uint32_t nc, uint32_t nr,
                const uint32_t* rec) {
    for (uint32_t k = 0; k < nc + nr; ++k) {
        const uint32_t n = k < nc ? w : h, base = k < nc ? 0u : w, u = list[k];
        const uint32_t* r = rec + 8u * k;
        if (!chk(r[0] == u && u < n, "fix-up record %u names %u, its list %u", k, r[0], u)) return false;
        const uint32_t nb[3] = {u ? u - 1u : 0u, u, std::min(u + 1u, n - 1u)};
        for (int t = 0; t < 3; ++t)
            if (!chk(r[1 + 2 * t] == plan[2u * (base + nb[t])] && r[2 + 2 * t] == plan[2u * (base + nb[t]) + 1u],
                     "fix-up record %u: plan entry %u differs", k, nb[t]))
                return false;
    }
    return true;
}
// The inexact columns of a same-size plan (its list's column count)
uint32_t n_inexact(uint32_t w, const uint32_t* plan) {
    uint32_t n = 0;
    for (uint32_t x = 0; x < w; ++x) n += plan[2u * x + 1u] != 0u;
    return n;
}
// The column records' word 7: 1 + the column's strip column (fixup_gather_kernel's qx)
bool strip_records_ok(const uint32_t* list, uint32_t nc, const uint32_t* stc, const uint32_t* rec) {
    for (uint32_t k = 0; k < nc; ++k)
        if (!chk(rec[8u * k + 7u] == stc[list[k]], "fix-up record %u: strip column %u, table %u", k, rec[8u * k + 7u], stc[list[k]]))
            return false;
    return true;
}
// The fix-up's column strips (bh_bloom_strip_table, up_sepq_kernel's STRIPS epilogue, fixup_gather_kernel):
// stc[c] is 0 or 1 + column c's strip column, distinct and below tw, so each strip word has one writer; and
// every texel a column lane of inexact column x reads (its own sample and F's at the sample's texels) lies in
// x's strip at the same offset: stc[c] - stc[x] == c - x.
bool strip_ok(uint32_t w, uint32_t h, const uint32_t* plan, const uint32_t* list, uint32_t nc, const uint32_t* stc,
              uint32_t tw) {
    if (!chk(tw > 0u && tw <= w && nc <= w, "strips: %u strip columns, %u inexact columns of %u", tw, nc, w)) return false;
    std::vector<uint8_t> seen(tw, 0u);
    for (uint32_t c = 0; c < w; ++c) {
        if (stc[c] == 0u) continue;
        const uint32_t q = stc[c] - 1u;
        if (!chk(q < tw && !seen[q], "strip table: column %u -> strip column %u of %u", c, q, tw)) return false;
        seen[q] = 1u;
    }
    for (uint32_t k = 0; k < nc; ++k) {
        const uint32_t x = list[k];
        if (!chk(x < w && stc[x] != 0u, "strips: inexact column %u outside every strip", x)) return false;
        auto same_strip = [&](uint32_t c) { return c < w && stc[c] != 0u && (int64_t)stc[c] - stc[x] == (int64_t)c - x; };
        const uint32_t e = plan[2u * x], ex = plan[2u * x + 1u];
        const uint32_t px[2] = {e & 0xFFFFu, e >> 16};
        for (int t = 0; t < (ex != 0u ? 2 : 1); ++t) {
            const uint32_t ep = plan[2u * px[t]], wp = plan[2u * px[t] + 1u];
            if (!chk(same_strip(px[t]) && same_strip(ep & 0xFFFFu) && (wp == 0u || same_strip(ep >> 16)),
                     "strips: column %u reads texel %u (samples %u, %u) outside its strip", x, px[t], ep & 0xFFFFu, ep >> 16))
                return false;
        }
    }
    (void)h;
    return true;
}
}  // namespace

// The strip table of a same-size plan's nc inexact columns (list, ascending): the columns within 2 of an
// inexact column, merged into contiguous runs (inexact columns cluster), numbered left to right: stc[c] = 1 +
// c's strip column, 0 outside.  Returns the number of strip columns (0: no inexact column).
extern "C" __attribute__((visibility("hidden"))) uint32_t bh_bloom_strip_table(uint32_t w, const uint32_t* list, uint32_t nc,
                                                                             uint32_t* stc) {
    std::fill(stc, stc + w, 0u);
    uint32_t tw = 0;
    for (uint32_t k = 0; k < nc; ++k) {
        const int64_t lo = std::max<int64_t>((int64_t)list[k] - 2, 0), hi = std::min<int64_t>((int64_t)list[k] + 2, (int64_t)w - 1);
        for (int64_t c = lo; c <= hi; ++c)
            if (stc[c] == 0u) stc[c] = ++tw;
    }
    return tw;
}

// The fix-up records of a list of n_cols columns then n_rows rows into out (8 words per entry, see
// fixup_gather_kernel).
extern "C" __attribute__((visibility("hidden"))) void bh_bloom_fixup_records(uint32_t w, uint32_t h, const uint32_t* plan,
                                                                           const uint32_t* list, uint32_t nc, uint32_t nr,
                                                                           uint32_t* out) {
    for (uint32_t k = 0; k < nc + nr; ++k) {
        const uint32_t n = k < nc ? w : h, base = k < nc ? 0u : w, u = std::min(list[k], n - 1u);
        const uint32_t nb[3] = {u ? u - 1u : 0u, u, std::min(u + 1u, n - 1u)};
        uint32_t* r = out + 8u * k;
        r[0] = list[k];
        for (int t = 0; t < 3; ++t) {
            r[1 + 2 * t] = plan[2u * (base + nb[t])];
            r[2 + 2 * t] = plan[2u * (base + nb[t]) + 1u];
        }
        r[7] = 0u;
    }
}

// The quad grid's origin for the in-block fix of a same-size plan (bh_bloom_same_plan): per axis the even
// offset in [0, 32) with the fewest inexact columns (rows) whose sample crosses a block edge (ties: the
// smallest), as org = ox | oy << 16; the crossing ones into cols / rows when given.  An offset may add a
// column (row) of blocks: at 1920 x 1080 offset 8 (61 block columns, no residual) measured 0.1234 ms per
// chain against 0.1265 for offset 0 (60 columns and a fix-up launch over the one crossing column)
// (profiles/r05/bloom_org/).  BH_BLOOM_ORG_KEEP (A/B): only offsets that keep the block count.
extern "C" __attribute__((visibility("hidden"))) uint32_t bh_bloom_same_org(uint32_t w, uint32_t h, const uint32_t* plan,
                                                                          std::vector<uint32_t>* cols,
                                                                          std::vector<uint32_t>* rows,
                                                                          std::vector<uint32_t>* cols2,
                                                                          std::vector<uint32_t>* rows2) {
    static const bool grow = std::getenv("BH_BLOOM_ORG_KEEP") == nullptr;
    uint32_t org = 0;
    for (int axis = 0; axis < 2; ++axis) {
        const uint32_t n = axis ? h : w, base = axis ? w : 0u;
        // fewest crossings of the final epilogue's fix (reach 2), then of the Y epilogue's, then the offset
        uint64_t best_n = UINT64_MAX;
        uint32_t best = 0;
        const uint32_t blocks = (n + 31u) / 32u;
        for (uint32_t off = 0; off < 32u && best_n != 0u; off += 2u) {
            if ((n + off + 31u) / 32u != blocks && !grow) break;  // offsets only grow the count
            uint64_t c2 = 0, c1 = 0;
            for (uint32_t x = 0; x < n; ++x) {
                c2 += same_crosses(plan, base, x, off, true) ? 1u : 0u;
                c1 += same_crosses(plan, base, x, off) ? 1u : 0u;
            }
            if ((c2 << 32 | c1) < best_n) { best_n = c2 << 32 | c1; best = off; }
        }
        org |= best << (axis ? 16 : 0);
        for (int r = 0; r < 2; ++r) {
            std::vector<uint32_t>* out = r ? (axis ? rows2 : cols2) : (axis ? rows : cols);
            if (!out) continue;
            out->clear();
            for (uint32_t x = 0; x < n; ++x)
                if (same_crosses(plan, base, x, best, r == 1)) out->push_back(x);
        }
    }
    return org;
}

// whether bh_launch_bloom_sep runs a plan of these extents with the quad kernel (the in-block fix's form)
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_sep_fix_ok(int ext, uint32_t ow, uint32_t oh, uint32_t epi);

// The separable up pass's launch form for a plan's extents (low 16 bits: 16x16 blocks, high: 32x32): the
// quad kernel when its footprint fits a 28 / 40 / 60 tile, else the one-pixel kernel at 24 / 44, else none
// (FP 0: the general pass).  One definition for the launcher and its check.
struct SepForm {
    int FP = 0, FS = 0;
    bool quad = false, raw = false;
};
static const bool g_no_sepq = std::getenv("BH_BLOOM_NO_SEPQ") != nullptr;  // A/B: the one-pixel kernel
static uint32_t env_u32(const char* name) {
    const char* e = std::getenv(name);
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 0u;
}
static SepForm sep_form(int ext, uint32_t ow, uint32_t oh) {
    // A/B: BH_BLOOM_SEPQ_MIN_BLOCKS=n runs a pass of fewer than n quad blocks (32x32 pixels) with the
    // one-pixel kernel (four times the blocks) when its footprint fits; BH_BLOOM_SEPQ_RAW bit 0 / bit 1
    // stage the 28 / 40 tiles as raw words too (decoded per read)
    static const uint32_t min_blocks = env_u32("BH_BLOOM_SEPQ_MIN_BLOCKS"), raw_mask = env_u32("BH_BLOOM_SEPQ_RAW");
    const int e16 = ext & 0xFFFF, e32 = (ext >> 16) & 0xFFFF;
    const int one = e16 <= 0 ? 0 : e16 <= 24 ? 24 : e16 <= 44 ? 44 : 0;
    int q = g_no_sepq || e32 <= 0 ? 0 : e32 <= 28 ? 28 : e32 <= 40 ? 40 : e32 <= 60 ? 60 : 0;
    const uint64_t qblocks = (uint64_t)((ow + 31u) / 32u) * ((oh + 31u) / 32u);
    if (qblocks < min_blocks && one != 0) q = 0;
    SepForm f;
    if (q != 0) {
        f.quad = true;
        f.FP = q;
        f.raw = q == 60 || (q == 28 && (raw_mask & 1u)) || (q == 40 && (raw_mask & 2u));
        f.FS = f.raw ? (q == 60 ? SEPQ_FS60 : 48) : (q == 28 ? 32 : 40);
    } else if (one != 0) {
        f.FP = one;
        f.raw = one == 44;
        f.FS = f.raw ? sep_stride<44, true>() : sep_stride<24, false>();
    }
    return f;
}

// A/B: BH_BLOOM_CAP_<PLAIN|Y|FINAL>=n caps the quad pass of that epilogue at n blocks per CU (dynamic LDS
// padding): a launch of 1.33 rounds of resident waves may finish sooner as 2 full rounds of less contended ones
static size_t sepq_cap_pad(const void* fn, uint32_t epi) {
    static const int cap[3] = {(int)env_u32("BH_BLOOM_CAP_PLAIN"), (int)env_u32("BH_BLOOM_CAP_Y"),
                               (int)env_u32("BH_BLOOM_CAP_FINAL")};
    const int n = epi < 3u ? cap[epi] : 0;
    if (n <= 0) return 0;
    hipFuncAttributes at{};
    if (hipFuncGetAttributes(&at, fn) != hipSuccess) return 0;
    const long want = 163840L / (n + 1) + 1 - (long)at.sharedSizeBytes;  // n + 1 blocks no longer fit
    return want > 0 ? (size_t)want : 0;
}

// whether bh_launch_bloom_sep runs a plan of these extents with epilogue epi in the in-block fix form: the
// quad kernel, and for the final epilogue a tile large enough for its words (sepq_fix2_fits)
static bool sep_fix_form(const SepForm& f, uint32_t epi) {
    if (!f.quad) return false;
    if (epi == EPI_Y) return true;
    const size_t tile = (f.raw ? 4u : 16u) * (size_t)(f.FP * f.FS + f.FP / 2);
    return epi == EPI_FINAL && tile >= 3u * FIX_WORDS * 4u;
}
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_sep_fix_ok(int ext, uint32_t ow, uint32_t oh, uint32_t epi) {
    return sep_fix_form(sep_form(ext, ow, oh), epi);
}

// bh_bloom_sep_plan's plan (host copy `plan`, extents `ext`) checked for the form bh_launch_bloom_sep takes:
// false (and the reason in *why) when any block's footprint exceeds its tile or any read leaves it.
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_sep_verify(uint32_t ow, uint32_t oh, uint32_t tw,
                                                                        uint32_t th, uint32_t rx, uint32_t ry,
                                                                        const uint32_t* plan, int ext, uint32_t org, bool fix,
                                                                        std::string* why) {
    std::string* prev = g_why;
    g_why = why;
    const SepForm f = sep_form(ext, ow, oh);
    const SepEntry* e = reinterpret_cast<const SepEntry*>(plan);
    const uint32_t B = f.quad ? 32u : 16u;
    const int size = f.quad ? f.FP * f.FS + f.FP / 2 : f.FP * f.FS;
    // the one-pixel kernel has no grid origin and no in-block fix
    const uint32_t ox = f.quad ? org & 0xFFFFu : 0u, oy = f.quad ? org >> 16 : 0u;
    const bool own = fix && f.quad;
    // FP == 0: no staged form fits these extents, and the launcher refuses the plan (the general pass runs)
    const bool ok = f.FP == 0 || (tile_ok(f.FP, f.FS, f.quad ? 1 : 0, size) && sep_axis_ok(e, ow, tw, rx, 0, B, f.FP, ox, own) &&
                                  sep_axis_ok(e + 8u * (size_t)ow, oh, th, ry, 1, B, f.FP, oy, own));
    g_why = prev;
    return ok;
}
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_same_verify(uint32_t w, uint32_t h, const uint32_t* plan,
                                                                         uint32_t nc, uint32_t nr, std::string* why) {
    std::string* prev = g_why;
    g_why = why;
    const bool ok = same_ok(w, h, plan, plan + 2u * ((size_t)w + h), nc, nr);
    g_why = prev;
    return ok;
}
// The fix-up records of a list (records_ok) and, when stc != nullptr, the column strips of the plan's full list
// with the column records' word 7 (strip_ok, strip_records_ok): what bh_bloom_check's dry run checks at each
// launch, run by sep_plan on every real plan before it is uploaded.
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_records_verify(uint32_t w, uint32_t h, const uint32_t* plan,
                                                                            const uint32_t* list, uint32_t nc, uint32_t nr,
                                                                            const uint32_t* rec, const uint32_t* stc,
                                                                            uint32_t strip_w, std::string* why) {
    std::string* prev = g_why;
    g_why = why;
    const bool ok = records_ok(w, h, plan, list, nc, nr, rec) &&
                    (!stc || (strip_ok(w, h, plan, list, nc, stc, strip_w) && strip_records_ok(list, nc, stc, rec)));
    g_why = prev;
    return ok;
}
// Dry mode (bh_bloom_check): while it is on, the launchers below check their launch's form on the host and
// return without launching; the plan pointers they receive are host copies.
extern "C" __attribute__((visibility("hidden"))) void bh_bloom_dry_begin(void) {
    delete g_dry;
    g_dry = new DryRun();
}
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_dry_end(uint64_t* launches, uint64_t* checks,
                                                                     std::string* fail, std::string* plan) {
    if (!g_dry) return false;
    if (launches) *launches = g_dry->launches;
    if (checks) *checks = g_dry->checks;
    if (fail) *fail = g_dry->fail;
    if (plan) *plan = g_dry->plan;
    const bool ok = g_dry->fail.empty();
    delete g_dry;
    g_dry = nullptr;
    return ok;
}
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_dry(void) { return g_dry != nullptr; }

// The separable plan of an 8-tap pass (see SepEntry / up_sep_kernel): 8 * (ow + oh) entries of 4 words
// into `outp` (per tap and column, then per tap and row), from the kernel's own f32 arithmetic: texcoord
// (x + 0.5) / n (the division core is IEEE division in its domain), the tap offset, sample_coord and
// floor.  Returns the largest 16x16 block footprint along either axis (the staged tile's side of
// up_sep_kernel) in the low 16 bits and the largest 32x32 block footprint (up_sepq_kernel, its grid at
// origin org) in the high ones, or -1 (texture sides above 65535).
extern "C" __attribute__((visibility("hidden"))) int bh_bloom_sep_plan(uint32_t ow, uint32_t oh, uint32_t tw,
                                                                     uint32_t th, uint32_t rx, uint32_t ry,
                                                                     uint32_t* outp, uint32_t org) {
    if (tw > 65535u || th > 65535u || tw == 0u || th == 0u || ow == 0u || oh == 0u) return -1;
    const float hx = 0.5f / (float)rx, hy = 0.5f / (float)ry;
    auto axis = [](uint32_t on, uint32_t tn, float d, uint32_t x, uint32_t* o) {
        const float t = h_sample_coord(((float)x + 0.5f) / (float)on + d, tn);
        const float f = floorf(t), fa = t - f, ia = 1.0f - fa;
        const int32_t fi = (int32_t)f;
        std::memcpy(&o[0], &fi, 4);
        std::memcpy(&o[1], &fa, 4);
        std::memcpy(&o[2], &ia, 4);
        o[3] = 0u;
    };
    auto fl = [&](size_t e) { int32_t v; std::memcpy(&v, outp + 4u * e, 4); return v; };
    for (int i = 0; i < 8; ++i) {
        const float du = (hx * (float)((int)((0x12343210u >> (4 * i)) & 15u) - 2)) * 3.0f;
        const float dv = (hy * (float)((int)((0x10123432u >> (4 * i)) & 15u) - 2)) * 3.0f;
        for (uint32_t x = 0; x < ow; ++x) axis(ow, tw, du, x, outp + 4u * ((size_t)i * ow + x));
        for (uint32_t y = 0; y < oh; ++y) axis(oh, th, dv, y, outp + 4u * (8u * (size_t)ow + (size_t)i * oh + y));
    }
    int ext[2] = {0, 0};  // 16- and 32-pixel blocks
    for (int q = 0; q < 2; ++q) {
        const uint32_t B = q ? 32u : 16u;
        for (int ax = 0; ax < 2; ++ax) {
            const uint32_t n = ax ? oh : ow;
            const size_t base = ax ? 8u * (size_t)ow : 0u;
            const int64_t off = q ? (ax ? org >> 16 : org & 0xFFFFu) : 0;
            for (int64_t bs = -off; bs < (int64_t)n; bs += B) {
                const uint32_t b = (uint32_t)std::max<int64_t>(bs, 0);
                const uint32_t l = (uint32_t)std::min<int64_t>(bs + B - 1, (int64_t)n - 1);
                int32_t lo = INT_MAX, hi = INT_MIN;
                for (int i = 0; i < 8; ++i) {
                    lo = std::min(lo, fl(base + (size_t)i * n + b));
                    hi = std::max(hi, fl(base + (size_t)i * n + l));
                }
                ext[q] = std::max(ext[q], hi - lo + 2);
            }
        }
    }
    return std::min(ext[0], 0x7FFF) | std::min(ext[1], 0x7FFF) << 16;  // up_sep_kernel's | up_sepq_kernel's
}

extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_sep(const float* lut, const float* enc,
                                                                        const uint8_t* buckets, const uint32_t* codes,
                                                                        const uint32_t* a, uint32_t aw, uint32_t ah,
                                                                        uint32_t rx, uint32_t ry,
                                                                        const uint32_t* sep, int ext, uint32_t epi,
                                                                        const uint32_t* own0, const uint32_t* own1,
                                                                        const uint32_t* same, uint32_t* out, uint32_t* aux,
                                                                        uint32_t ow, uint32_t oh, uint32_t org, bool fix,
                                                                        const uint32_t* stc, uint32_t* strips,
                                                                        uint32_t strip_w, bool* strips_written,
                                                                        hipStream_t s) {
    if (strips_written) *strips_written = false;
    const SepForm f = sep_form(ext, ow, oh);
    if (f.FP == 0 || !sep) return (int)hipErrorInvalidValue;
    // the grid origin and the in-block fix are the quad kernel's (the fix with the Y or final epilogue)
    if (!f.quad) org = 0u;
    fix = fix && sep_fix_form(f, epi);
    // the fix-up's column strips: the quad kernel's final epilogue without its in-block fix
    const bool st = stc && f.quad && epi == EPI_FINAL && !fix && same;
    if (g_dry) {  // the plan is a host copy: check the form's every read instead of launching
        char form[32];
        std::snprintf(form, sizeof form, "%s%d%s/%u%s", f.quad ? "sepq" : "sep", f.FP, f.raw ? "r" : "", epi, fix ? "f" : "");
        note_launch(form, ow, oh, aw, ah, rx, ry);
        if (st && !strip_ok(ow, oh, same, same + 2u * ((size_t)ow + oh), n_inexact(ow, same), stc, strip_w))
            return (int)hipErrorInvalidValue;
        if (strips_written) *strips_written = st;
        return bh_bloom_sep_verify(ow, oh, aw, ah, rx, ry, sep, ext, org, fix, nullptr) &&
                       (epi == EPI_PLAIN || chk(same != nullptr, "separable epilogue without a same-size plan"))
                   ? 0
                   : (int)hipErrorInvalidValue;
    }
    if (st && !strips) return (int)hipErrorInvalidValue;
    const uint32_t* const STC = st ? stc : nullptr;
    const Tables tb{lut, enc, buckets, codes};
    const CTex A{a, aw, ah}, O0{own0 ? own0 : a, ow, oh}, O1{own1 ? own1 : a, ow, oh};
    const SepEntry* P = reinterpret_cast<const SepEntry*>(sep);
    const uint2* S = reinterpret_cast<const uint2*>(same);
    const Tex O{out, ow, oh}, X{aux ? aux : out, ow, oh};
    const dim3 g = grid_for(ow, oh), gq((ow + (org & 0xFFFFu) + 31u) / 32u, (oh + (org >> 16) + 31u) / 32u);
#define BH_SEP(FP, E, RAW) \
    hipLaunchKernelGGL((up_sep_kernel<FP, E, RAW>), g, dim3(256), 0, s, tb, A, rx, ry, P, O, O0, O1, S, X)
#define BH_SEPQ(FP, E, RAW, FS, FX)                                                                                  \
    do {                                                                                                             \
        hipLaunchKernelGGL((up_sepq_kernel<FP, E, RAW, FS, FX>), gq, dim3(256),                                      \
                           sepq_cap_pad(reinterpret_cast<const void*>(&up_sepq_kernel<FP, E, RAW, FS, FX>), E), s, tb, A, \
                           rx, ry, P, O, O0, O1, S, X, org, STC, strips, strip_w);                                   \
    } while (0)
#define BH_EPI(LAUNCH, ...)                                                    \
    do {                                                                       \
        if (epi == EPI_Y) LAUNCH(__VA_ARGS__, EPI_Y, _);                       \
        else if (epi == EPI_FINAL && fix) LAUNCH(__VA_ARGS__, EPI_FINAL, true); \
        else if (epi == EPI_FINAL) LAUNCH(__VA_ARGS__, EPI_FINAL, _);          \
        else LAUNCH(__VA_ARGS__, EPI_PLAIN, _);                                \
    } while (0)
#define BH_Q(FPv, RAWv, FSv, E, FX) BH_SEPQ(FPv, E, RAWv, FSv, BH_FIX_##FX)
#define BH_FIX_true true
#define BH_FIX__ false
#define BH_1(FPv, RAWv, E, _) BH_SEP(FPv, E, RAWv)
    // the instantiations sep_form can name (its FS follows from FP and raw)
    if (f.quad && f.FP == 28 && f.raw) BH_EPI(BH_Q, 28, true, 48);
    else if (f.quad && f.FP == 40 && f.raw) BH_EPI(BH_Q, 40, true, 48);
    else if (f.quad && f.FP == 28) BH_EPI(BH_Q, 28, false, 32);
    else if (f.quad && f.FP == 40) BH_EPI(BH_Q, 40, false, 40);
    else if (f.quad && f.FP == 60) BH_EPI(BH_Q, 60, true, SEPQ_FS60);
    else if (f.FP == 24) BH_EPI(BH_1, 24, false);
    else if (f.FP == 44) BH_EPI(BH_1, 44, true);
    else return (int)hipErrorInvalidValue;
#undef BH_1
#undef BH_FIX_true
#undef BH_FIX__
#undef BH_Q
#undef BH_EPI
#undef BH_SEPQ
#undef BH_SEP
    const hipError_t e = hipGetLastError();
    if (strips_written) *strips_written = st && e == hipSuccess;
    return (int)e;
}

// The fix-up pass of a fused epilogue (fixup_kernel): `list` = n_cols columns then n_rows rows
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_fixup(const float* lut, const float* enc,
                                                                          const uint8_t* buckets, const uint32_t* codes,
                                                                          uint32_t epi, const uint32_t* a, const uint32_t* b,
                                                                          const uint32_t* c, const uint32_t* same,
                                                                          const uint32_t* list, uint32_t n_cols,
                                                                          uint32_t n_rows, uint32_t* out, uint32_t w,
                                                                          uint32_t h, int32_t residual_org, const uint32_t* recs,
                                                                          const uint32_t* stc, const uint32_t* strips,
                                                                          uint32_t strip_w, hipStream_t s) {
    if (n_cols > w || n_rows > h || !list || !same) return (int)hipErrorInvalidValue;  // the list of this frame's plan
    // the column strips (the full list of the final epilogue, with its records; stc: the table they were written by)
    static const bool no_rec = std::getenv("BH_BLOOM_FIXUP_NOREC") != nullptr;  // A/B: list, then plan
    const bool st = stc && recs && !no_rec && epi == EPI_FINAL && residual_org < 0;
    const uint64_t n = (uint64_t)n_cols * h + (uint64_t)n_rows * w;
    if (g_dry) {
        // residual_org < 0: the list of every inexact column and row, right after the plan; else the residual
        // list of the in-block fix at that grid origin (crossing columns and rows only)
        note_launch(residual_org < 0 ? (epi == EPI_Y ? "fixup/1" : "fixup/2") : (epi == EPI_Y ? "fixup/1r" : "fixup/2r"), w, h,
                    n_cols, n_rows, 0u, 0u);
        const bool ok = residual_org < 0
                            ? same_ok(w, h, same, list, n_cols, n_rows) &&
                                  chk(list == same + 2u * ((size_t)w + h), "fix-up list is not its plan's")
                            : same_ok(w, h, same, nullptr, 0u, 0u, false) &&
                                  residual_ok(w, h, same, list, n_cols, n_rows, (uint32_t)residual_org, epi == EPI_FINAL);
        return ok && (!recs || records_ok(w, h, same, list, n_cols, n_rows, recs)) &&
                       (!st || (strip_ok(w, h, same, list, n_cols, stc, strip_w) && strip_records_ok(list, n_cols, stc, recs)))
                   ? 0
                   : (int)hipErrorInvalidValue;
    }
    if (st && !strips) return (int)hipErrorInvalidValue;
    const uint32_t* const SP = st ? strips : nullptr;
    if (n == 0) return 0;
    const Tables tb{lut, enc, buckets, codes};
    const dim3 g0((uint32_t)((n + 255u) / 256u));
    const uint2* S = reinterpret_cast<const uint2*>(same);
    static const bool per_sample = std::getenv("BH_BLOOM_FIXUP_SAMPLE") != nullptr;  // A/B: the per-sample form
    const uint4* R = no_rec ? nullptr : reinterpret_cast<const uint4*>(recs);
    const dim3 g = g0;
    if (!per_sample && epi == EPI_Y)
        hipLaunchKernelGGL(fixup_gather_kernel<EPI_Y>, g, dim3(256), 0, s, tb, CTex{a, w, h}, CTex{b, w, h},
                           CTex{b, w, h}, S, list, n_cols, n_rows, Tex{out, w, h}, R, nullptr, 0u);
    else if (!per_sample)
        hipLaunchKernelGGL(fixup_gather_kernel<EPI_FINAL>, g, dim3(256), 0, s, tb, CTex{a, w, h}, CTex{b, w, h},
                           CTex{c, w, h}, S, list, n_cols, n_rows, Tex{out, w, h}, R, SP, strip_w);
    else if (epi == EPI_Y)
        hipLaunchKernelGGL(fixup_kernel<EPI_Y>, g, dim3(256), 0, s, tb, CTex{a, w, h}, CTex{b, w, h}, CTex{b, w, h}, S, list,
                           n_cols, n_rows, Tex{out, w, h});
    else
        hipLaunchKernelGGL(fixup_kernel<EPI_FINAL>, g, dim3(256), 0, s, tb, CTex{a, w, h}, CTex{b, w, h}, CTex{c, w, h}, S,
                           list, n_cols, n_rows, Tex{out, w, h});
    return (int)hipGetLastError();
}

// Two downsamples a -> (mw x mh) -> out in one pass (down2_kernel); false: not taken (BH_BLOOM_NO_DOWN2,
// A/B), the caller runs the two passes
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_down2(const float* lut, const float* enc,
                                                                          const uint8_t* buckets, const uint32_t* codes,
                                                                          const uint32_t* a, uint32_t aw, uint32_t ah,
                                                                          uint32_t mw, uint32_t mh, uint32_t* out,
                                                                          uint32_t ow, uint32_t oh, hipStream_t s) {
    if (mw == 0u || mh == 0u) return (int)hipErrorInvalidValue;
    if (g_dry) {  // every index of down2_kernel is clamped to its texture (down_at): only the sizes to check
        note_launch("down2", ow, oh, aw, ah, mw, mh);
        return chk(aw > 0u && ah > 0u && ow > 0u && oh > 0u, "down2 of an empty texture") ? 0 : (int)hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(down2_kernel, grid_for(ow, oh), dim3(256), 0, s, Tables{lut, enc, buckets, codes}, CTex{a, aw, ah},
                       mw, mh, Tex{out, ow, oh});
    return (int)hipGetLastError();
}

// The same-size plan of a w x h frame (remix_plan_kernel): per column, then per row, the two clamped
// texels and the weight of a sample at the pixel's own texcoord ((x + 0.5) / n, sample_coord, floor).
// Texel indices are 16-bit fields: w, h <= 65536.
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_same_plan(uint32_t w, uint32_t h, uint32_t* outp) {
    if (w > 65536u || h > 65536u || w == 0u || h == 0u) return false;
    auto axis = [](uint32_t n, uint32_t x, uint32_t* o) {
        const float t = h_sample_coord(((float)x + 0.5f) / (float)n, n);
        const float f = floorf(t), wgt = t - f;
        const int32_t hi = (int32_t)n - 1;
        const int32_t a0 = std::min(std::max((int32_t)f, 0), hi), a1 = std::min(std::max((int32_t)f + 1, 0), hi);
        o[0] = (uint32_t)a0 | (uint32_t)a1 << 16;
        std::memcpy(&o[1], &wgt, 4);
    };
    for (uint32_t x = 0; x < w; ++x) axis(w, x, outp + 2u * x);
    for (uint32_t y = 0; y < h; ++y) axis(h, y, outp + 2u * ((size_t)w + y));
    return true;
}

extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_remix_plan(const float* lut, const float* enc,
                                                                               const uint8_t* buckets,
                                                                               const uint32_t* codes, const uint32_t* a,
                                                                               const uint32_t* b, const uint32_t* plan,
                                                                               uint32_t* out, uint32_t w, uint32_t h,
                                                                               hipStream_t s) {
    if (g_dry) {  // the plan's texel indices (host copy)
        note_launch("remix_plan", w, h, w, h, w, h);
        return chk(plan != nullptr, "remix without a plan") && same_ok(w, h, plan, nullptr, 0u, 0u, false) ? 0
                                                                                                                : (int)hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(remix_plan_kernel, grid_for(w, h), dim3(256), 0, s, Tables{lut, enc, buckets, codes},
                       CTex{a, w, h}, CTex{b, w, h}, reinterpret_cast<const uint2*>(plan), Tex{out, w, h});
    return (int)hipGetLastError();
}
// same_copy_kernel: out = the copy pass of src (and of the blur's same-size down: the same sample)
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_same_copy(const float* lut, const float* enc,
                                                                              const uint8_t* buckets,
                                                                              const uint32_t* codes, const uint32_t* src,
                                                                              const uint32_t* plan, uint32_t* out,
                                                                              uint32_t w, uint32_t h, hipStream_t s) {
    if (g_dry) {  // the plan's texel indices (host copy)
        note_launch("same_copy", w, h, w, h, w, h);
        return chk(plan != nullptr, "same-size copy without a plan") && same_ok(w, h, plan, nullptr, 0u, 0u, false)
                   ? 0
                   : (int)hipErrorInvalidValue;
    }
    const dim3 g((w + 63u) / 64u, (h + 4u * SAME_COPY_ROWS - 1u) / (4u * SAME_COPY_ROWS));
    hipLaunchKernelGGL(same_copy_kernel, g, dim3(256), 0, s, Tables{lut, enc, buckets, codes}, CTex{src, w, h},
                       reinterpret_cast<const uint2*>(plan), Tex{out, w, h});
    return (int)hipGetLastError();
}
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_remix2_plan(const float* lut, const float* enc,
                                                                                const uint8_t* buckets,
                                                                                const uint32_t* codes,
                                                                                const uint32_t* col, const uint32_t* Y,
                                                                                const uint32_t* Bt, const uint32_t* plan,
                                                                                uint32_t* out, uint32_t w, uint32_t h,
                                                                                hipStream_t s) {
    if (g_dry) {  // the plan's texel indices (host copy)
        note_launch("remix2_plan", w, h, w, h, w, h);
        return chk(plan != nullptr, "remix without a plan") && same_ok(w, h, plan, nullptr, 0u, 0u, false) ? 0
                                                                                                       : (int)hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(remix2_plan_kernel, grid_for(w, h), dim3(256), 0, s, Tables{lut, enc, buckets, codes},
                       CTex{col, w, h}, CTex{Y, w, h}, CTex{Bt, w, h}, reinterpret_cast<const uint2*>(plan),
                       Tex{out, w, h});
    return (int)hipGetLastError();
}

// bit i: tap i of kawase_upsample.wgsl samples texel centres exactly for every pixel of an
// ow x oh pass over a tw x th texture with resolution uniform (rx, ry)
extern "C" __attribute__((visibility("hidden"))) uint32_t bh_bloom_point_mask(uint32_t ow, uint32_t oh, uint32_t tw,
                                                                             uint32_t th, uint32_t rx, uint32_t ry) {
    const float hx = 0.5f / (float)rx, hy = 0.5f / (float)ry;
    uint32_t m = 0;
    for (int i = 0; i < 8; ++i) {
        const float du = (hx * (float)((int)((0x12343210u >> (4 * i)) & 15u) - 2)) * 3.0f;
        const float dv = (hy * (float)((int)((0x10123432u >> (4 * i)) & 15u) - 2)) * 3.0f;
        if (axis_point(ow, tw, du) && axis_point(oh, th, dv)) m |= 1u << i;
    }
    return m;
}

// Whether bh_launch_bloom_pass runs an up pass of this shape with up_sep_kernel (neither the TapPlan nor
// the Up2Plan form applies): only then does the host build the shape's separable plan (bh_bloom_sep_plan).
static const bool g_no_up2 = std::getenv("BH_BLOOM_NO_UP2") != nullptr;  // A/B: the general up pass
static const bool g_no_sep = std::getenv("BH_BLOOM_NO_SEP") != nullptr;  // A/B: the per-pixel sampler
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_up_uses_sep(uint32_t ow, uint32_t oh, uint32_t aw,
                                                                         uint32_t ah, uint32_t rx, uint32_t ry) {
    if (g_no_sep || tap_plan(ow, oh, aw, ah, rx, ry).valid) return false;
    return g_no_up2 || !up2_plan(ow, oh, aw, ah, rx, ry).valid;
}

extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_pass(uint32_t shader, const float* lut,
                                                                         const float* enc, const uint8_t* buckets,
                                                                         const uint32_t* codes, const uint32_t* a,
                                                                         uint32_t aw, uint32_t ah, const uint32_t* b,
                                                                         uint32_t rx, uint32_t ry, uint32_t* out,
                                                                         uint32_t ow, uint32_t oh, const uint32_t* sep,
                                                                         int sep_ext, hipStream_t s) {
    const Tables tb{lut, enc, buckets, codes};
    const CTex A{a, aw, ah}, B{b ? b : a, aw, ah};
    const Tex O{out, ow, oh};
    const TapPlan P = shader == SH_UP ? tap_plan(ow, oh, aw, ah, rx, ry) : TapPlan{};
    const uint32_t pm = shader == SH_UP && !P.valid && !g_dry ? bh_bloom_point_mask(ow, oh, aw, ah, rx, ry) : 0u;
    if (shader == SH_UP && !P.valid && !g_no_up2) {
        const Up2Plan Q = up2_plan(ow, oh, aw, ah, rx, ry);
        if (Q.valid && g_dry) {
            note_launch(std_up2_plan(Q) == 12 ? "up2_12" : std_up2_plan(Q) == 3 ? "up2_3" : "up2_0", ow, oh, aw, ah, rx, ry);
            const bool ok = tile_ok(FP_UPQ, FS_UPQ, 0, FP_UPQ * FS_UPQ) && up2_axis_ok(Q, ow, aw, rx, 0, FP_UPQ) &&
                            up2_axis_ok(Q, oh, ah, ry, 1, FP_UPQ);
            return ok ? 0 : (int)hipErrorInvalidValue;
        }
        if (Q.valid) {
            const dim3 g((ow + 31u) / 32u, (oh + 31u) / 32u);
            switch (std_up2_plan(Q)) {
                case 12: hipLaunchKernelGGL(up2_kernel<12>, g, dim3(256), 0, s, tb, A, rx, ry, pm, Q, O); break;
                case 3: hipLaunchKernelGGL(up2_kernel<3>, g, dim3(256), 0, s, tb, A, rx, ry, pm, Q, O); break;
                default: hipLaunchKernelGGL(up2_kernel<0>, g, dim3(256), 0, s, tb, A, rx, ry, pm, Q, O); break;
            }
            return (int)hipGetLastError();
        }
    }
    if (shader == SH_UP && !P.valid && sep && sep_form(sep_ext, ow, oh).FP != 0 && !g_no_sep) {
        return bh_launch_bloom_sep(lut, enc, buckets, codes, a, aw, ah, rx, ry, sep, sep_ext, EPI_PLAIN, nullptr, nullptr,
                                   nullptr, out, nullptr, ow, oh, 0u, false, nullptr, nullptr, 0u, nullptr, s);
    }
    if (g_dry) {  // pass_kernel: an up pass stages through with_source<FP_UP>; the others read clamped indices
        note_launch(shader == SH_UP ? (P.valid ? "pass_up_tap" : "pass_up") : shader == SH_COPY ? "pass_copy"
                    : shader == SH_DOWN ? "pass_down" : "pass_remix", ow, oh, aw, ah, rx, ry);
        const bool ok = chk(aw > 0u && ah > 0u && ow > 0u && oh > 0u, "pass over an empty texture") &&
                        (shader != SH_UP || (tile_ok(FP_UP, FP_UP, 0, FP_UP * FP_UP) &&
                                             tapplan_axis_ok(P, ow, aw, rx, 0, 16u, FP_UP) &&
                                             tapplan_axis_ok(P, oh, ah, ry, 1, 16u, FP_UP)));
        return ok ? 0 : (int)hipErrorInvalidValue;
    }
    switch (shader) {
        case SH_COPY: hipLaunchKernelGGL(pass_kernel<SH_COPY>, grid_for(ow, oh), dim3(256), 0, s, tb, A, B, rx, ry, pm, P, O); break;
        case SH_DOWN: hipLaunchKernelGGL(pass_kernel<SH_DOWN>, grid_for(ow, oh), dim3(256), 0, s, tb, A, B, rx, ry, pm, P, O); break;
        case SH_UP: hipLaunchKernelGGL(pass_kernel<SH_UP>, grid_for(ow, oh), dim3(256), 0, s, tb, A, B, rx, ry, pm, P, O); break;
        default: hipLaunchKernelGGL(pass_kernel<SH_REMIX>, grid_for(ow, oh), dim3(256), 0, s, tb, A, B, rx, ry, pm, P, O); break;
    }
    return (int)hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_down2_fusable(uint32_t w, uint32_t h) {
    // the sides multiples of 32 (the Y quad kernel's block: every lane inside the frame), and down2_kernel's
    // sample arithmetic (down_at) on every pixel of both levels: texel 2 x' and 2 x' + 1, weight 0.5 -- which
    // holds at powers of two, not at display sizes such as 1920 x 1080 (37 and 32 inexact samples per axis)
    auto axis = [](uint32_t n) {
        if (n % 32u != 0u) return false;
        for (uint32_t on = n / 2u, tn = n; on >= n / 4u; tn = on, on /= 2u)
            for (uint32_t x = 0; x < on; ++x) {
                const float t = h_sample_coord(h_texcoord(x, on), tn), f = floorf(t);
                if (f != (float)(2u * x) || t - f != 0.5f || 2u * x + 1u > tn - 1u) return false;
            }
        return true;
    };
    return axis(w) && axis(h);
}

extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_y(const float* lut, const float* enc,
                                                                      const uint8_t* buckets, const uint32_t* codes,
                                                                      const uint32_t* X, uint32_t* Y, uint32_t w,
                                                                      uint32_t h, uint32_t* d2out, bool* d2_done,
                                                                      hipStream_t s) {
    const TapPlan P = tap_plan(w, h, w, h, w, h);
    static const bool no_quad = std::getenv("BH_BLOOM_NO_YQUAD") != nullptr;  // A/B: one pixel per lane
    static const bool no_yd2 = std::getenv("BH_BLOOM_NO_YDOWN2") != nullptr;  // A/B: down2_kernel after the Y pass
    const bool quad = P.valid && !no_quad && P.hi_x - P.lo_x + 32 <= FP_YQ && P.hi_y - P.lo_y + 32 <= FP_YQ;
    const bool d2 = quad && d2out && !no_yd2 && bh_bloom_down2_fusable(w, h);
    if (d2_done) *d2_done = d2;
    if (g_dry) {  // the quad form's tile (row-pair shift) or with_source<FP_Y>
        note_launch(quad ? (std_tap_plan(P) == 12 ? "yq12" : "yq0") : "y1", w, h, w, h, w, h);
        if (d2) note_launch("down2f", w / 4u, h / 4u, w, h, w / 2u, h / 2u);  // fused into the Y launch
        const bool ok = quad ? tile_ok(FP_YQ, FS_YQ, 2, FP_YQ * FS_YQ + FP_YQ / 2 + 1) &&
                                   tapplan_axis_ok(P, w, w, w, 0, 32u, FP_YQ) && tapplan_axis_ok(P, h, h, h, 1, 32u, FP_YQ)
                             : tile_ok(FP_Y, FP_Y, 0, FP_Y * FP_Y) && tapplan_axis_ok(P, w, w, w, 0, 16u, FP_Y) &&
                                   tapplan_axis_ok(P, h, h, h, 1, 16u, FP_Y);
        return ok ? 0 : (int)hipErrorInvalidValue;
    }
    if (quad) {
        const dim3 g((w + 31u) / 32u, (h + 31u) / 32u);
        const Tables tb{lut, enc, buckets, codes};
        const Tex D{d2 ? d2out : Y, w / 4u, h / 4u};
        if (std_tap_plan(P) == 12 && d2)
            hipLaunchKernelGGL((bloom_yq_kernel<12, true>), g, dim3(256), 0, s, tb, CTex{X, w, h}, P, Tex{Y, w, h}, D);
        else if (std_tap_plan(P) == 12)
            hipLaunchKernelGGL((bloom_yq_kernel<12, false>), g, dim3(256), 0, s, tb, CTex{X, w, h}, P, Tex{Y, w, h}, D);
        else if (d2)
            hipLaunchKernelGGL((bloom_yq_kernel<0, true>), g, dim3(256), 0, s, tb, CTex{X, w, h}, P, Tex{Y, w, h}, D);
        else
            hipLaunchKernelGGL((bloom_yq_kernel<0, false>), g, dim3(256), 0, s, tb, CTex{X, w, h}, P, Tex{Y, w, h}, D);
        return (int)hipGetLastError();
    }
    const uint32_t pm = P.valid ? 0u : bh_bloom_point_mask(w, h, w, h, w, h);
    hipLaunchKernelGGL(bloom_y_kernel, grid_for(w, h), dim3(256), 0, s, Tables{lut, enc, buckets, codes}, CTex{X, w, h}, pm, P,
                       Tex{Y, w, h});
    return (int)hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_final(const float* lut, const float* enc,
                                                                          const uint8_t* buckets, const uint32_t* codes,
                                                                          const uint32_t* col, const uint32_t* Y,
                                                                          const uint32_t* U0, uint32_t rx, uint32_t ry,
                                                                          uint32_t* out, uint32_t w, uint32_t h,
                                                                          hipStream_t s) {
    const TapPlan P = tap_plan(w, h, w, h, rx, ry);
    if (g_dry) {  // with_source<FP_FINAL>: the TapPlan form (raw words) or the span fallback
        note_launch(P.valid ? (std_tap_plan(P) == 48 ? "final48" : "final0") : "final", w, h, w, h, rx, ry);
        const bool ok = tile_ok(FP_FINAL, FP_FINAL, 0, FP_FINAL * FP_FINAL) &&
                        tapplan_axis_ok(P, w, w, rx, 0, 16u, FP_FINAL) && tapplan_axis_ok(P, h, h, ry, 1, 16u, FP_FINAL);
        return ok ? 0 : (int)hipErrorInvalidValue;
    }
    const uint32_t pm = P.valid ? 0u : bh_bloom_point_mask(w, h, w, h, rx, ry);
    // the kernel's with_source takes the TapPlan form exactly when this holds (raw words staged)
    const bool plan = P.valid && P.hi_x - P.lo_x + 16 <= FP_FINAL && P.hi_y - P.lo_y + 16 <= FP_FINAL;
    const size_t lds = (size_t)FP_FINAL * FP_FINAL * (plan ? sizeof(uint32_t) : sizeof(float4));
    const bool std48 = plan && std_tap_plan(P) == 48;
    // persistent blocks: measured no faster; BH_BLOOM_PERSIST=1 takes them (A/B)
    static const bool persist = std::getenv("BH_BLOOM_PERSIST") != nullptr;
    const uint32_t tiles_x = (w + 15u) / 16u, n_tiles = tiles_x * ((h + 15u) / 16u);
    const uint32_t G = persistent_grid(7u);
    if (std48 && persist && n_tiles >= 2u * G)
        hipLaunchKernelGGL(bloom_final_pkernel<48>, dim3(G), dim3(256), 0, s, Tables{lut, enc, buckets, codes},
                           CTex{col, w, h}, CTex{Y, w, h}, CTex{U0, w, h}, P, Tex{out, w, h}, tiles_x, n_tiles);
    else if (std48)
        hipLaunchKernelGGL(bloom_final_kernel<48>, grid_for(w, h), dim3(256), lds, s, Tables{lut, enc, buckets, codes},
                           CTex{col, w, h}, CTex{Y, w, h}, CTex{U0, w, h}, rx, ry, pm, P, Tex{out, w, h});
    else
        hipLaunchKernelGGL(bloom_final_kernel<0>, grid_for(w, h), dim3(256), lds, s, Tables{lut, enc, buckets, codes},
                           CTex{col, w, h}, CTex{Y, w, h}, CTex{U0, w, h}, rx, ry, pm, P, Tex{out, w, h});
    return (int)hipGetLastError();
}
