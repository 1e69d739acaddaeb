// Micro-benchmark of VALU issue rates on gfx950 (tools only; guides the march kernel design).
// Each kernel runs ITER iterations of an unrolled body; reports ns and cycles per wave-instruction
// per SIMD assuming the measured clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <chrono>

#define ITER 2048
template <int CHAINS>
__global__ void k_fma(float* out, float a, float b) {
    float x[CHAINS];
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < ITER; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_fmaf(x[c], a, b);
    }
    float s = 0; for (int c = 0; c < CHAINS; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
template <int CHAINS>
__global__ void k_div(float* out, float a, float b) {   // correctly rounded division (compiler expansion)
    float x[CHAINS];
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.f;
    for (int i = 0; i < ITER; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = a / x[c] + b;
    }
    float s = 0; for (int c = 0; c < CHAINS; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
template <int CHAINS>
__global__ void k_rcp(float* out, float a, float b) {
    float x[CHAINS];
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.f;
    for (int i = 0; i < ITER; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_amdgcn_rcpf(x[c]) + b;
    }
    float s = 0; for (int c = 0; c < CHAINS; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
template <int CHAINS>
__global__ void k_sqrt(float* out, float a, float b) {  // correctly rounded sqrt (compiler expansion)
    float x[CHAINS];
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.f;
    for (int i = 0; i < ITER; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_sqrtf(x[c]) + b;
    }
    float s = 0; for (int c = 0; c < CHAINS; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
template <int CHAINS>
__global__ void k_pkfma(float* out, float a, float b) {
    typedef float float2_t __attribute__((ext_vector_type(2)));
    float2_t x[CHAINS];
    float2_t av = {a, a}, bv = {b, b};
    for (int c = 0; c < CHAINS; ++c) { x[c].x = threadIdx.x * 1e-3f + c; x[c].y = x[c].x + 1; }
    for (int i = 0; i < ITER; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_elementwise_fma(x[c], av, bv);
    }
    float s = 0; for (int c = 0; c < CHAINS; ++c) s += x[c].x + x[c].y;
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <typename K>
double timeit(K kern, float* out, int blocks, int threads) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001f, 1e-7f);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001f, 1e-7f);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / 5.0;
}

int main() {
    float* out; hipMalloc(&out, 1 << 20);
    int cus; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const double clk = 2.4e9;
    // 8 waves per SIMD: 256-thread blocks, 8 per CU
    int blocks = cus * 8, threads = 256;
    double waves_per_simd = 8.0;
#define RUN(name, K, ops_per_iter) { double ms = timeit(K, out, blocks, threads); \
    double instr = (double)ITER * ops_per_iter * waves_per_simd; \
    printf("%-22s %8.3f ms  %6.2f cyc/wave-instr/SIMD (@2.4GHz)\n", name, ms, ms * 1e-3 * clk / instr); }
    RUN("fma  1 chain", k_fma<1>, 1); RUN("fma  4 chains", k_fma<4>, 4); RUN("fma 16 chains", k_fma<16>, 16);
    RUN("pkfma 1 chain", k_pkfma<1>, 1); RUN("pkfma 8 chains", k_pkfma<8>, 8);
    RUN("rcp  1 chain (+add)", k_rcp<1>, 2); RUN("rcp  8 chains (+add)", k_rcp<8>, 16);
    RUN("CRdiv 1 chain (+add)", k_div<1>, 1); RUN("CRdiv 4 chains (+add)", k_div<4>, 4);
    RUN("CRsqrt 1 chain (+add)", k_sqrt<1>, 1); RUN("CRsqrt 4 chains (+add)", k_sqrt<4>, 4);
    // 4 waves per SIMD
    blocks = cus * 4; waves_per_simd = 4.0;
    RUN("fma  1 chain  4w", k_fma<1>, 1); RUN("fma  4 chains 4w", k_fma<4>, 4);
    RUN("CRdiv 4 chains 4w", k_div<4>, 4);
    blocks = cus * 1; waves_per_simd = 1.0;
    RUN("fma  1 chain  1w", k_fma<1>, 1); RUN("fma 16 chains 1w", k_fma<16>, 16);
    return 0;
}
