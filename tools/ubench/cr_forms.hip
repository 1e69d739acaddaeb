// cr_forms.hip — exhaustive checks of shorter correctly rounded f32 sqrt / division forms on gfx950.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         tools/ubench/cr_forms.hip -o tools/ubench/cr_forms
//
// S: sqrt_rsq(x) = fma(x - s*s, y/2, s) with y = v_rsq(x), s = x*y, against IEEE sqrt over EVERY
//    non-negative float; mismatches are histogrammed by biased exponent (the domain to guard).
// R: rcp_refined(d) = fma(1 - d*r0, r0, r0) against IEEE 1/d over every positive normal float.
// D: div1(n, d) = fma(-(d*y - n), r, y) with y = n*r (ONE residual correction) against the two-
//    correction div_core of bh_crmath.hpp, over EVERY pair of significands n, d in [1, 2) (2^46
//    pairs).  Every op is exactly scale-covariant in the guarded normal range (checked for v_rcp by
//    R's exponent histogram and op X below), so the [1, 2)^2 square covers the whole domain.
// X: v_rcp scale covariance: rcp(m * 2^e) == rcp(m) * 2^-e for every m in [1, 2), e in [-40, 60].
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__device__ __forceinline__ float sqrt_rsq(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y;
    const float h = 0.5f * y;
    const float r = __builtin_fmaf(-s, s, x);
    return __builtin_fmaf(r, h, s);
}
__device__ __forceinline__ float rcp_ref(float d) {
    const float r = __builtin_amdgcn_rcpf(d);
    return __builtin_fmaf(__builtin_fmaf(-d, r, 1.0f), r, r);
}

__global__ void k_sqrt(uint32_t lo, uint32_t hi, unsigned long long* hist, uint32_t* ex) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; (uint64_t)lo + i <= hi; i += stride) {
        const uint32_t b = lo + (uint32_t)i;
        const float x = __uint_as_float(b);
        const float got = sqrt_rsq(x), want = __builtin_sqrtf(x);
        if (__float_as_uint(got) != __float_as_uint(want)) {
            const unsigned long long k = atomicAdd(&hist[b >> 23], 1ull);
            if (k == 0) ex[b >> 23] = b;
        }
    }
}
__global__ void k_rcp(unsigned long long* hist, uint32_t* ex) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 0x7F000000ull; i += stride) {
        const uint32_t b = 0x00800000u + (uint32_t)i;
        const float d = __uint_as_float(b);
        const float got = rcp_ref(d), want = 1.0f / d;
        if (__float_as_uint(got) != __float_as_uint(want)) {
            const unsigned long long k = atomicAdd(&hist[b >> 23], 1ull);
            if (k == 0) ex[b >> 23] = b;
        }
    }
}
__global__ void k_rcpscale(unsigned long long* cnt) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;   // 2^23 significands
    if (m >= (1u << 23)) return;
    const float d1 = __uint_as_float(0x3F800000u | m);
    const uint32_t r1 = __float_as_uint(__builtin_amdgcn_rcpf(d1)), q1 = __float_as_uint(rcp_ref(d1));
    for (int e = -40; e <= 60; ++e) {
        const float d = __uint_as_float((uint32_t)(127 + e) << 23 | m);
        const uint32_t r = __float_as_uint(__builtin_amdgcn_rcpf(d)), q = __float_as_uint(rcp_ref(d));
        if (r + ((uint32_t)e << 23) != r1 || q + ((uint32_t)e << 23) != q1) atomicAdd(cnt, 1ull);
    }
}
// pairs: d significand = blockIdx-major, n significands in [n0, n0 + nspan)
// cnt[0]: div1(refined r) != div_core; cnt[1]: div_core with UNREFINED r0 != div_core;
// cnt[2]: div_core != IEEE (sampled: every 64th wave-chunk of n)
__global__ void __launch_bounds__(256) k_div(uint32_t d0, uint32_t n0, uint32_t nspan, unsigned long long* cnt,
                                             uint32_t* ex) {
    const uint32_t dm = d0 + blockIdx.y;
    const float d = __uint_as_float(0x3F800000u | dm);
    const float r0 = __builtin_amdgcn_rcpf(d);
    const float r = __builtin_fmaf(__builtin_fmaf(-d, r0, 1.0f), r0, r0);
    uint32_t c0 = 0, c1 = 0, c2 = 0;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nspan; j += gridDim.x * blockDim.x) {
        const uint32_t nb = 0x3F800000u | (n0 + j);
        const float n = __uint_as_float(nb);
        const float y = n * r;
        const float e1 = __builtin_fmaf(d, y, -n);
        const float y1 = __builtin_fmaf(-e1, r, y);
        const float e2 = __builtin_fmaf(d, y1, -n);
        const float q = __builtin_fmaf(-e2, r, y1);
        // unrefined reciprocal, two corrections
        const float z = n * r0;
        const float f1 = __builtin_fmaf(d, z, -n);
        const float z1 = __builtin_fmaf(-f1, r0, z);
        const float f2 = __builtin_fmaf(d, z1, -n);
        const float zq = __builtin_fmaf(-f2, r0, z1);
        if (__float_as_uint(y1) != __float_as_uint(q)) {
            ++c0;
            if (atomicAdd(&cnt[3], 1ull) < 4) { uint32_t k = atomicAdd((uint32_t*)&cnt[4], 1u); if (k < 4) { ex[2*k] = nb; ex[2*k+1] = __float_as_uint(d); } }
        }
        if (__float_as_uint(zq) != __float_as_uint(q)) ++c1;
        if (((j >> 6) & 63u) == 0u && __float_as_uint(n / d) != __float_as_uint(q)) ++c2;
    }
    if (c0) atomicAdd(&cnt[0], (unsigned long long)c0);
    if (c1) atomicAdd(&cnt[1], (unsigned long long)c1);
    if (c2) atomicAdd(&cnt[2], (unsigned long long)c2);
}

static void hist_print(const char* name, unsigned long long* dh, uint32_t* dex) {
    unsigned long long h[256]; uint32_t e[256];
    hipMemcpy(h, dh, sizeof h, hipMemcpyDeviceToHost); hipMemcpy(e, dex, sizeof e, hipMemcpyDeviceToHost);
    unsigned long long tot = 0;
    for (int i = 0; i < 256; ++i) tot += h[i];
    printf("%s: %llu mismatches\n", name, tot);
    for (int i = 0; i < 256; ++i)
        if (h[i]) printf("  biased exp %3d (2^%d): %llu  e.g. 0x%08x\n", i & 255, (i & 255) - 127, h[i], e[i]);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int div_slices = argc > 1 ? atoi(argv[1]) : 64;   // of 2^23 d significands; 64 = all
    unsigned long long* hist; uint32_t* ex; unsigned long long* cnt;
    hipMalloc(&hist, 256 * 8); hipMalloc(&ex, 256 * 4); hipMalloc(&cnt, 8 * 8);
    hipMemset(hist, 0, 256 * 8); hipMemset(ex, 0, 256 * 4);
    k_sqrt<<<8192, 256>>>(0u, 0x7F800000u, hist, ex);
    hipDeviceSynchronize();
    hist_print("S sqrt_rsq vs IEEE sqrt (x in [0, inf])", hist, ex);
    hipMemset(hist, 0, 256 * 8); hipMemset(ex, 0, 256 * 4);
    k_rcp<<<8192, 256>>>(hist, ex);
    hipDeviceSynchronize();
    hist_print("R rcp_refined vs IEEE 1/d (normal d)", hist, ex);
    hipMemset(cnt, 0, 8 * 8);
    k_rcpscale<<<(1u << 23) / 256, 256>>>(cnt);
    unsigned long long hc[8];
    hipMemcpy(hc, cnt, 8 * 8, hipMemcpyDeviceToHost);
    printf("X rcp / rcp_refined scale covariance violations (e in [-40, 60]): %llu\n", hc[0]);
    fflush(stdout);
    hipMemset(cnt, 0, 8 * 8); hipMemset(ex, 0, 256 * 4);
    const uint32_t per = (1u << 23) / 64;
    hipEvent_t t0, t1; hipEventCreate(&t0); hipEventCreate(&t1);
    for (int s = 0; s < div_slices; ++s) {
        hipEventRecord(t0);
        for (uint32_t dd = 0; dd < per; dd += 1024)   // 1024 d's x 2^23 n's per launch
            k_div<<<dim3(64, 1024), 256>>>(s * per + dd, 0u, 1u << 23, cnt, ex);
        hipEventRecord(t1); hipEventSynchronize(t1);
        float ms = 0; hipEventElapsedTime(&ms, t0, t1);
        hipMemcpy(hc, cnt, 8 * 8, hipMemcpyDeviceToHost);
        printf("D slice %2d/%d (%.0f ms): div1 != div_core %llu | unrefined-rcp div_core != div_core %llu | div_core != IEEE (1/64 sampled) %llu\n",
               s + 1, div_slices, ms, hc[0], hc[1], hc[2]);
        fflush(stdout);
    }
    uint32_t e[8];
    hipMemcpy(e, ex, sizeof e, hipMemcpyDeviceToHost);
    for (int k = 0; k < 4 && k < (int)hc[3]; ++k) printf("  div1 example n=0x%08x d=0x%08x\n", e[2*k], e[2*k+1]);
    return 0;
}
