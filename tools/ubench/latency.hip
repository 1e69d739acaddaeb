// Dependent-chain issue model on gfx950: C independent FMA chains per wave, W waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 1024
template <int C>
__global__ void __launch_bounds__(256) k(float* out, float a, float b) {
    float x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < ITER; ++i) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = __builtin_fmaf(x[c], a, b);
        }
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
template <int C>
void run(float* out, int cus, int waves_per_simd) {
    int blocks = cus * waves_per_simd;  // 256-thread blocks = 4 waves = one per SIMD
    hipLaunchKernelGGL(k<C>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001f, 1e-7f);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<C>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001f, 1e-7f);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
    double instr = (double)ITER * 16 * C * waves_per_simd;  // wave-instructions per SIMD
    printf("chains %2d  waves/SIMD %d : %7.3f ms  %6.2f ns/instr/SIMD  %5.2f cyc@2.2GHz\n", C, waves_per_simd, ms,
           ms * 1e6 / instr, ms * 1e-3 * 2.2e9 / instr);
}
int main() {
    float* out; hipMalloc(&out, 1 << 20);
    int cus; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int w : {1, 2, 4, 8}) { run<1>(out, cus, w); run<2>(out, cus, w); run<4>(out, cus, w); run<8>(out, cus, w); }
    return 0;
}
