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

#ifndef BH_FAST
#error "define BH_FAST to 0 or 1"
#endif

namespace bh {
namespace BH_NS {

struct v3 { float x, y, z; };

__device__ __forceinline__ v3 mk(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 smul(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
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

__device__ __forceinline__ uint32_t texel_u32(const MarchArgs& a, int32_t x, int32_t y) {
    return a.sky[(size_t)y * a.sky_w + (size_t)x];
}
__device__ __forceinline__ v3 decode(const float* lut, uint32_t t) {
    return mk(lut[t & 0xffu], lut[(t >> 8) & 0xffu], lut[(t >> 16) & 0xffu]);
}
__device__ __forceinline__ int32_t clampi(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

// textureSampleLevel(t_diffuse, s_diffuse, uv, 0) on Rgba8UnormSrgb, mag=Linear, clamp-to-edge
// (src/texture.rs:41,62-70): decode texels, then bilinear with fp32 weights.
__device__ __forceinline__ v3 sample_sky(const MarchArgs& a, const float* lut, float u, float v) {
    if (u != u || v != v) return decode(lut, texel_u32(a, 0, 0));  // Q8
    float tx = u * (float)a.sky_w - 0.5f;
    float ty = v * (float)a.sky_h - 0.5f;
    tx = fminf(fmaxf(tx, -1.0f), (float)a.sky_w);
    ty = fminf(fmaxf(ty, -1.0f), (float)a.sky_h);
    float fx0 = floorf(tx), fy0 = floorf(ty);
    float fa = tx - fx0, fb = ty - fy0;
    int32_t x0 = (int32_t)fx0, y0 = (int32_t)fy0;
    const int32_t wm = (int32_t)a.sky_w - 1, hm = (int32_t)a.sky_h - 1;
    int32_t x1 = clampi(x0 + 1, 0, wm), y1 = clampi(y0 + 1, 0, hm);
    x0 = clampi(x0, 0, wm);
    y0 = clampi(y0, 0, hm);
    v3 t00 = decode(lut, texel_u32(a, x0, y0)), t10 = decode(lut, texel_u32(a, x1, y0));
    v3 t01 = decode(lut, texel_u32(a, x0, y1)), t11 = decode(lut, texel_u32(a, x1, y1));
    float ia = 1.0f - fa, ib = 1.0f - fb;
    v3 top = add(muls(t00, ia), muls(t10, fa));
    v3 bot = add(muls(t01, ia), muls(t11, fa));
    return add(muls(top, ib), muls(bot, fb));
}

// get_col (:259-345)
__device__ __forceinline__ Ray get_col(const MarchArgs& a, const float* lut, v3 ro0, v3 rd0) {
    v3 ro = ro0, rd = rd0;
    v3 c = cross(ro, rd);                                   // :262
    const float h2 = dot(c, c);                             // :263
    const float s = ((a.dp * a.rs) * -1.5f) * h2;           // :126 scalar chain, loop-invariant
    const v3 nro0 = normalize(ro0);
    const v3 cps = muls(muls(mk(-nro0.x, -nro0.y, -nro0.z), 1.5f), a.rs);  // :294
    float travelled = 0.0f;                                 // :264
    bool outside = false;                                   // :265
    Ray out;
    out.fate = BH_FATE_CAP;
    uint32_t i = 0;
    for (; i < a.max_iters; ++i) {                          // :266
        const float r = len(ro);                            // :271
        if (a.blackout_eh != 0u) {                          // :272-283
            if (r < 1.0f && dot(rd, ro) < 0.0f) { out.fate = BH_FATE_BLACKOUT; break; }
            if (r > 1.0f) outside = true;
            else if (outside) { out.fate = BH_FATE_BLACKOUT; break; }
        }
        const float ds = sdf(ro, a.rs, a.scene_flags);      // :285
        if (ds < MIN_DIST) { out.fate = BH_FATE_SURFACE; break; }  // :286-288
        const float dps = len(sub(cps, ro)) - 0.075f;       // :294
        const float dist = fminf(ds, dps);                  // :299
        const float dd = fminf(dist * 0.9f, a.dtm * r);     // :307-310
        // get_delta_photon_rk4 (:134-151)
        const float dt = dd;
        v3 ro_k1 = smul(dt, rd);
        v3 rd_k1 = smul(dt, accel(ro, s));
        v3 ro_k2 = smul(dt, add(rd, smul(0.5f, rd_k1)));
        v3 rd_k2 = smul(dt, accel(add(ro, smul(0.5f, ro_k1)), s));
        v3 ro_k3 = smul(dt, add(rd, smul(0.5f, rd_k2)));
        v3 rd_k3 = smul(dt, accel(add(ro, smul(0.5f, ro_k2)), s));
        v3 ro_k4 = smul(dt, add(rd, rd_k3));
        v3 rd_k4 = smul(dt, accel(add(ro, ro_k3), s));
#if BH_FAST
        constexpr float SIXTH = 1.0f / 6.0f;
        v3 dro = muls(add(add(add(ro_k1, smul(2.0f, ro_k2)), smul(2.0f, ro_k3)), ro_k4), SIXTH);
        v3 drd = muls(add(add(add(rd_k1, smul(2.0f, rd_k2)), smul(2.0f, rd_k3)), rd_k4), SIXTH);
#else
        v3 dro = divs(add(add(add(ro_k1, smul(2.0f, ro_k2)), smul(2.0f, ro_k3)), ro_k4), 6.0f);
        v3 drd = divs(add(add(add(rd_k1, smul(2.0f, rd_k2)), smul(2.0f, rd_k3)), rd_k4), 6.0f);
#endif
        ro = add(ro, dro);                                  // :315
        rd = add(rd, drd);                                  // :322
        travelled += dd;                                    // :324
        if (travelled > a.max_dist) { ++i; out.fate = BH_FATE_ESCAPE; break; }  // :325-327
    }
    out.n_rk = i;
    if (out.fate == BH_FATE_BLACKOUT) { out.col = mk(0.0f, 0.0f, 0.0f); return out; }
    if (out.fate == BH_FATE_SURFACE) { out.col = mk(1.0f, 1.0f, 1.0f); return out; }
    const v3 n = normalize(rd);                             // :330
#if BH_FAST
    const float az = atan2f(n.z, n.x);                      // :332
#else
    const float az = (float)atan2((double)n.z, (double)n.x);
#endif
    const float x = (az + ONE_PI) / TWO_PI;                 // :334
    const float y = (n.y + 1.0f) * 0.5f;                    // :336
    v3 col = sample_sky(a, lut, x, 1.0f - y);               // :341
#if BH_FAST
    col.y = col.y * __builtin_sqrtf(col.y);                 // :342
    col.z = col.z * __builtin_sqrtf(col.z);                 // :343
#else
    col.y = pow15(col.y);
    col.z = pow15(col.z);
#endif
    out.col = col;
    return out;
}

__device__ __forceinline__ void store_px(void* base, uint32_t fmt, size_t idx, v3 c) {
    if (fmt == BH_OUT_RGBA32F) {
        reinterpret_cast<float4*>(base)[idx] = make_float4(c.x, c.y, c.z, 1.0f);
    } else if (fmt == BH_OUT_RGBA16F) {
        __half2 lo = __floats2half2_rn(c.x, c.y);
        __half2 hi = __floats2half2_rn(c.z, 1.0f);
        uint2 w;
        w.x = *reinterpret_cast<uint32_t*>(&lo);
        w.y = *reinterpret_cast<uint32_t*>(&hi);
        reinterpret_cast<uint2*>(base)[idx] = w;
    }
}

// One wave64 = one 8x8 tile; 4 waves (4 tiles) per 256-thread workgroup.
__global__ void __launch_bounds__(256) march_kernel(MarchArgs a) {
    __shared__ float lut[256];
    lut[threadIdx.x] = a.srgb_lut[threadIdx.x];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t t = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (t >= a.n_tiles) return;
    uint32_t tx, ty;
    shard_tile_coords(t, a.tiles_x, a.shard_index, a.shard_count, &tx, &ty);
    const uint32_t px = tx * 8u + (lane & 7u), py = ty * 8u + (lane >> 3);
    if (px >= a.width || py >= a.height) return;

    // vs_main + rasteriser interpolation + fs_main :362 (screen triangle (3,1),(-1,1),(-1,-3))
    const float l0 = ((float)px + 0.5f) / (2.0f * (float)a.width);
    const float l2 = ((float)py + 0.5f) / (2.0f * (float)a.height);
    const float l1 = (1.0f - l0) - l2;
    const v3 d = add(add(smul(l0, mk(a.c0[0], a.c0[1], a.c0[2])), smul(l1, mk(a.c1[0], a.c1[1], a.c1[2]))),
                     smul(l2, mk(a.c2[0], a.c2[1], a.c2[2])));
    const v3 ro0 = mk(a.pos[0], a.pos[1], a.pos[2]);
    const Ray ray = get_col(a, lut, ro0, normalize(d));

    const size_t idx = (a.layout == BH_LAYOUT_TILES) ? (size_t)t * 64u + lane : (size_t)py * a.width + px;
    store_px(a.out_col, a.format, idx, ray.col);
    if (a.out_blackout) {                                   // :365-368
        const v3 bo = dot(ray.col, ray.col) < 1.0f ? mk(0.0f, 0.0f, 0.0f) : ray.col;
        store_px(a.out_blackout, a.format, idx, bo);
    }
    if (a.dbg_n_rk) a.dbg_n_rk[idx] = (uint16_t)ray.n_rk;
    if (a.dbg_fate) a.dbg_fate[idx] = (uint8_t)ray.fate;
}

}  // namespace BH_NS
}  // namespace bh
