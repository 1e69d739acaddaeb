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
// HBM-bound byte work: one lane per output pixel, 4-byte texel gathers (L2-resident neighbourhoods),
// coalesced 4-byte stores; the 256-entry decode table and the 257 encode thresholds in LDS.
#include <hip/hip_runtime.h>

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

// LDS tables of a block: sRGB decode (256), alpha decode k/255 (256), the encoder's thresholds (257)
// and base codes (table form, bh_srgb.hpp)
struct Lds {
    float lut[256], alut[256], T[SRGB_TABLE];
    uint32_t B32[SRGB_BUCKETS / 4];
};
struct Tables {
    const float* lut;      // 256
    const float* enc;      // 257
    const uint8_t* bkt;    // SRGB_BUCKETS
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

__device__ __forceinline__ F4 dec(const Lds& L, uint32_t t) {
    return {L.lut[(t >> 16) & 0xffu], L.lut[(t >> 8) & 0xffu], L.lut[t & 0xffu], L.alut[t >> 24]};
}
__device__ __forceinline__ int32_t clampi(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ uint32_t unorm8(float a) {
    if (!(a > 0.0f)) return 0u;
    if (a >= 1.0f) return 255u;
    return (uint32_t)__double2int_rd((double)a * 255.0 + 0.5);
}
// the Bgra8UnormSrgb store of a pass's result
__device__ __forceinline__ uint32_t enc(const Lds& L, F4 c) {
    const uint8_t* B = reinterpret_cast<const uint8_t*>(L.B32);
    return srgb_encode_lut(c.b, B, L.T) | (srgb_encode_lut(c.g, B, L.T) << 8) | (srgb_encode_lut(c.r, B, L.T) << 16) |
           (unorm8(c.a) << 24);
}
__device__ __forceinline__ F4 quant(const Lds& L, F4 c) { return dec(L, enc(L, c)); }

// Texcoord of pixel i of an n-pixel axis, (i + 0.5) / n: the correctly rounded division core with the
// reciprocal of n shared by the block (exact: n >= 1 and i + 0.5 >= 0.5 are inside its domain).
__device__ __forceinline__ float texcoord(uint32_t i, const crm::Rcp& R) { return crm::div_core((float)i + 0.5f, R); }

// x / 12 of the up-sampling filter: the div12 core where it is exact (x == 0 or |x| >= 2^-60,
// selftest op 5), IEEE division otherwise (never taken by sums of decoded texels).
__device__ __forceinline__ float div12(float x) {
    float q = crm::div12(x);
    if (__builtin_expect(crm::key(x) < crm::KEY_MIN, 0)) q = x / 12.0f;
    return q;
}

// Texel sources: decoded texel (x, y) of a BGRA8 texture straight from global memory, or from a
// block's LDS tile of pre-decoded texels covering exactly the footprint the block samples.
struct GlobalSrc {
    CTex t;
    const Lds* L;
    __device__ __forceinline__ F4 at(int32_t x, int32_t y) const { return dec(*L, t.px[(size_t)y * t.w + x]); }
};
template <int FP>
struct TileSrc {
    CTex t;
    const float4* tile;  // decoded texels [y0, y0 + FP) x [x0, x0 + FP)
    int32_t x0, y0;
    __device__ __forceinline__ F4 at(int32_t x, int32_t y) const {
        const float4 v = tile[(y - y0) * FP + (x - x0)];
        return {v.x, v.y, v.z, v.w};
    }
};

// clamp-to-edge bilinear of decoded texels at texcoord (u, v) (oracle: sample)
__device__ __forceinline__ float sample_coord(float u, uint32_t n) {
    const float t = u * (float)n - 0.5f;
    return fminf(fmaxf(t, -1.0f), (float)n);
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
        const F4 q = ((point >> i) & 1u) ? sample_point(src, tu, tv) : sample(src, tu, tv);
        const float w = (i & 1) ? 2.0f : 1.0f;  // x * 1.0 == x exactly: one form for both weights
        s.r = s.r + q.r * w; s.g = s.g + q.g * w; s.b = s.b + q.b * w; s.a = s.a + q.a * w;
    }
    return {div12(s.r), div12(s.g), div12(s.b), div12(s.a)};
}
// remix.wgsl:22-24
__device__ __forceinline__ F4 remix(F4 c0, F4 c1) {
    return {c0.r + c1.r * 0.5f, c0.g + c1.g * 0.5f, c0.b + c1.b * 0.5f, c0.a + c1.a * 0.5f};
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
// else straight from global memory; both give identical values.  Called by every thread.
template <int FP, class Body>
__device__ __forceinline__ void with_source(CTex t, const Lds& L, float4* tile, const Taps& k, uint32_t ow,
                                            uint32_t oh, const crm::Rcp& Rw, const crm::Rcp& Rh, Body body) {
    const uint32_t bx = blockIdx.x * 16u, by = blockIdx.y * 16u;
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
                raw[r] = t.px[(size_t)(sy.lo + ly) * t.w + (sx.lo + lx)];
            }
        }
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
        body(GlobalSrc{t, &L});
    }
}

#ifndef BH_BLOOM_WPE
#define BH_BLOOM_WPE 1
#endif
// occupancy floor for the 8-tap kernels: the unrolled taps otherwise take 160 VGPRs (3 waves/SIMD)
#define BLOOM_BOUNDS __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BH_BLOOM_WPE)))
constexpr int FP_UP = 24;     // staged footprint of a generic up pass (taps within a few texels)
constexpr int FP_Y = 24;      // blur1 at full size: taps within +-3 texels (22 x 22)
constexpr int FP_FINAL = 44;  // the last up pass at res / 4: taps within +-12 texels (42 x 42)

// One render pass of the reference (literal schedule): 16x16 pixels per 256-thread block.
template <uint32_t SH>
__global__ void BLOOM_BOUNDS pass_kernel(Tables tb, CTex a, CTex b, uint32_t rx, uint32_t ry, uint32_t point, Tex out) {
    __shared__ Lds L;
    __shared__ float4 tile[SH == SH_UP ? FP_UP * FP_UP : 1];
    load_tables(tb, L);
    const uint32_t x = blockIdx.x * 16u + (threadIdx.x & 15u), y = blockIdx.y * 16u + (threadIdx.x >> 4);
    const crm::Rcp Rw = crm::rcp_refined((float)out.w), Rh = crm::rcp_refined((float)out.h);
    if constexpr (SH == SH_UP) {
        const Taps k(rx, ry);
        with_source<FP_UP>(a, L, tile, k, out.w, out.h, Rw, Rh, [&](const auto& src) {
            if (x >= out.w || y >= out.h) return;
            out.px[(size_t)y * out.w + x] = enc(L, up8(src, k, texcoord(x, Rw), texcoord(y, Rh), point));
        });
    } else {
        if (x >= out.w || y >= out.h) return;
        const float u = texcoord(x, Rw), v = texcoord(y, Rh);
        const GlobalSrc A{a, &L};
        F4 r;
        if constexpr (SH == SH_COPY || SH == SH_DOWN) r = sample(A, u, v);
        else r = remix(sample(A, u, v), sample(GlobalSrc{b, &L}, u, v));
        out.px[(size_t)y * out.w + x] = enc(L, r);
    }
}

// Fused stage 1 (same-size sampling exact): Y = X + 0.5 * q(blur1(X)), blur1 = up8(X, res (W, H)).
__global__ void BLOOM_BOUNDS bloom_y_kernel(Tables tb, CTex X, uint32_t point, Tex Y) {
    __shared__ Lds L;
    __shared__ float4 tile[FP_Y * FP_Y];
    load_tables(tb, L);
    const uint32_t x = blockIdx.x * 16u + (threadIdx.x & 15u), y = blockIdx.y * 16u + (threadIdx.x >> 4);
    const crm::Rcp Rw = crm::rcp_refined((float)Y.w), Rh = crm::rcp_refined((float)Y.h);
    const Taps k(X.w, X.h);
    with_source<FP_Y>(X, L, tile, k, Y.w, Y.h, Rw, Rh, [&](const auto& src) {
        if (x >= Y.w || y >= Y.h) return;
        const F4 b1 = quant(L, up8(src, k, texcoord(x, Rw), texcoord(y, Rh), point));
        Y.px[(size_t)y * Y.w + x] = enc(L, remix(src.at((int32_t)x, (int32_t)y), b1));
    });
}

// Fused last stage: out = col + 0.5 * q(Z), Z = Y + 0.5 * q(up8(U0, res (rx, ry))).
__global__ void BLOOM_BOUNDS bloom_final_kernel(Tables tb, CTex col, CTex Y, CTex U0, uint32_t rx,
                                                   uint32_t ry, uint32_t point, Tex out) {
    __shared__ Lds L;
    __shared__ float4 tile[FP_FINAL * FP_FINAL];
    load_tables(tb, L);
    const uint32_t x = blockIdx.x * 16u + (threadIdx.x & 15u), y = blockIdx.y * 16u + (threadIdx.x >> 4);
    const crm::Rcp Rw = crm::rcp_refined((float)out.w), Rh = crm::rcp_refined((float)out.h);
    const Taps k(rx, ry);
    with_source<FP_FINAL>(U0, L, tile, k, out.w, out.h, Rw, Rh, [&](const auto& src) {
        if (x >= out.w || y >= out.h) return;
        const size_t i = (size_t)y * out.w + x;
        const F4 b3 = quant(L, up8(src, k, texcoord(x, Rw), texcoord(y, Rh), point));
        const F4 z = quant(L, remix(dec(L, Y.px[i]), b3));
        out.px[i] = enc(L, remix(dec(L, col.px[i]), z));
    });
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

extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_pass(uint32_t shader, const float* lut,
                                                                         const float* enc, const uint8_t* buckets,
                                                                         const uint32_t* a,
                                                                         uint32_t aw, uint32_t ah, const uint32_t* b,
                                                                         uint32_t rx, uint32_t ry, uint32_t* out,
                                                                         uint32_t ow, uint32_t oh, hipStream_t s) {
    const Tables tb{lut, enc, buckets};
    const CTex A{a, aw, ah}, B{b ? b : a, aw, ah};
    const Tex O{out, ow, oh};
    const uint32_t pm = shader == SH_UP ? bh_bloom_point_mask(ow, oh, aw, ah, rx, ry) : 0u;
    switch (shader) {
        case SH_COPY: hipLaunchKernelGGL(pass_kernel<SH_COPY>, grid_for(ow, oh), dim3(256), 0, s, tb, A, B, rx, ry, pm, O); break;
        case SH_DOWN: hipLaunchKernelGGL(pass_kernel<SH_DOWN>, grid_for(ow, oh), dim3(256), 0, s, tb, A, B, rx, ry, pm, O); break;
        case SH_UP: hipLaunchKernelGGL(pass_kernel<SH_UP>, grid_for(ow, oh), dim3(256), 0, s, tb, A, B, rx, ry, pm, O); break;
        default: hipLaunchKernelGGL(pass_kernel<SH_REMIX>, grid_for(ow, oh), dim3(256), 0, s, tb, A, B, rx, ry, pm, O); break;
    }
    return (int)hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_y(const float* lut, const float* enc,
                                                                      const uint8_t* buckets, const uint32_t* X, uint32_t* Y, uint32_t w,
                                                                      uint32_t h, hipStream_t s) {
    const uint32_t pm = bh_bloom_point_mask(w, h, w, h, w, h);
    hipLaunchKernelGGL(bloom_y_kernel, grid_for(w, h), dim3(256), 0, s, Tables{lut, enc, buckets}, CTex{X, w, h}, pm, Tex{Y, w, h});
    return (int)hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_final(const float* lut, const float* enc,
                                                                          const uint8_t* buckets, const uint32_t* col, const uint32_t* Y,
                                                                          const uint32_t* U0, uint32_t rx, uint32_t ry,
                                                                          uint32_t* out, uint32_t w, uint32_t h,
                                                                          hipStream_t s) {
    const uint32_t pm = bh_bloom_point_mask(w, h, w, h, rx, ry);
    hipLaunchKernelGGL(bloom_final_kernel, grid_for(w, h), dim3(256), 0, s, Tables{lut, enc, buckets}, CTex{col, w, h},
                       CTex{Y, w, h}, CTex{U0, w, h}, rx, ry, pm, Tex{out, w, h});
    return (int)hipGetLastError();
}
