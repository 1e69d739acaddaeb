// Micro-benchmark (tools only): does a transcendental (v_rcp_f32 / v_rsq_f32) hold the SIMD's vector
// issue for its whole 8 cycles, or can other waves' plain VALU issue beside it?  Kernels run a body of
// T independent rcp chains and F independent fma chains per iteration at 8 waves per SIMD; the
// cycles per iteration are compared with T*8 + F*2 (blocking) and max(T*8, (T+F)*2) (overlapped).
// The clock is measured inside the kernel (s_memtime / s_memrealtime), not assumed.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITER 4096
template <int T, int F, int RSQ>
__global__ void __launch_bounds__(256) k_mix(float* out, unsigned long long* clk, float a, float b) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float x[T > 0 ? T : 1], y[F > 0 ? F : 1];
#pragma unroll
    for (int c = 0; c < T; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.f;
#pragma unroll
    for (int c = 0; c < F; ++c) y[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < ITER; ++i) {
#pragma unroll
        for (int c = 0; c < (T > F ? T : F); ++c) {
            if (c < T) x[c] = RSQ ? __builtin_amdgcn_rsqf(x[c]) : __builtin_amdgcn_rcpf(x[c]);
            if (c < F) y[c] = __builtin_fmaf(y[c], a, b);
        }
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < T; ++c) s += x[c];
#pragma unroll
    for (int c = 0; c < F; ++c) s += y[c];
    if (s == 12345.f) out[threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <typename K>
void run(const char* name, K kern, float* out, unsigned long long* clk, int blocks, int T, int F) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, clk, 1.0000001f, 1e-7f);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    double best = 1e30, mhz = 0;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, clk, 1.0000001f, 1e-7f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned long long h[2];
        hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
        const double m = h[0] / (h[1] / 100.0);  // shader MHz seen by wave 0
        // the whole grid's cycles at that clock over 8 waves per SIMD, each ITER iterations
        const double cyc_per_iter = ms * 1e-3 * m * 1e6 / (8.0 * ITER);
        if (cyc_per_iter < best) { best = cyc_per_iter; mhz = m; }
    }
    printf("%-28s T=%d F=%d  %7.2f cyc/iter/SIMD  blocking %5.1f  overlapped %5.1f  (%.0f MHz)\n", name, T, F, best,
           T * 8.0 + F * 2.0, (T * 8.0 > (T + F) * 2.0 ? T * 8.0 : (T + F) * 2.0), mhz);
}

int main() {
    float* out; hipMalloc(&out, 1 << 20);
    unsigned long long* clk; hipMalloc(&clk, 64);
    int cus; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;
#define R(T, F, S) run(#T "rcp/rsq " #F "fma" #S, k_mix<T, F, S>, out, clk, blocks, T, F)
    R(0, 8, 0); R(0, 16, 0);
    R(4, 0, 0); R(8, 0, 0); R(4, 0, 1);
    R(1, 4, 0); R(1, 8, 0); R(2, 8, 0); R(4, 8, 0); R(4, 4, 0); R(2, 16, 0); R(1, 16, 0);
    R(1, 8, 1); R(2, 8, 1); R(4, 8, 1);
    return 0;
}
