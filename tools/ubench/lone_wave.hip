// What one wave ALONE on the GPU sustains (the frame's tail: a few capped rays march their serial
// step chains after the bulk has drained).  One 64-lane workgroup; s_memtime (shader clock) around
// an unrolled loop; cycles per wave-instruction for independent streams (issue cost) and dependent
// chains (latency), packed-FP32 included.  Tools only.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/lone_wave.hip -o /tmp/lone_wave && /tmp/lone_wave
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
#define N 4096

#define KERNEL(name, T, INIT, BODY, CHAINS)                                                    \
    __global__ void name(float* out, long long* cyc, float a, float b) {                       \
        T x[CHAINS];                                                                           \
        for (int c = 0; c < CHAINS; ++c) { INIT; }                                             \
        long long t0 = __builtin_amdgcn_s_memtime();                                           \
        for (int i = 0; i < N; ++i) {                                                          \
            _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) { BODY; }                        \
        }                                                                                      \
        long long t1 = __builtin_amdgcn_s_memtime();                                           \
        float s = 0;                                                                           \
        for (int c = 0; c < CHAINS; ++c) s += (float)x[c][0];                                  \
        out[threadIdx.x] = s;                                                                  \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                                \
    }

// scalar float wrapped as a 1-element "vector" so one macro serves both
struct S1 { float v; __device__ float& operator[](int) { return v; } };

KERNEL(fma_dep, S1, x[c].v = threadIdx.x * 1e-3f + c, x[c].v = __builtin_fmaf(x[c].v, a, b), 1)
KERNEL(fma_ind8, S1, x[c].v = threadIdx.x * 1e-3f + c, x[c].v = __builtin_fmaf(x[c].v, a, b), 8)
KERNEL(mul_dep, S1, x[c].v = threadIdx.x * 1e-3f + c + 1, x[c].v = x[c].v * a, 1)
KERNEL(add_dep, S1, x[c].v = threadIdx.x * 1e-3f + c, x[c].v = x[c].v + b, 1)
KERNEL(pkfma_dep, f2, (x[c] = f2{threadIdx.x * 1e-3f + c, 1.f + c}), x[c] = __builtin_elementwise_fma(x[c], (f2{a, a}), (f2{b, b})), 1)
KERNEL(pkfma_ind8, f2, (x[c] = f2{threadIdx.x * 1e-3f + c, 1.f + c}), x[c] = __builtin_elementwise_fma(x[c], (f2{a, a}), (f2{b, b})), 8)
KERNEL(pkmul_dep, f2, (x[c] = f2{threadIdx.x * 1e-3f + c + 1, 2.f + c}), x[c] = x[c] * (f2{a, a}), 1)
KERNEL(pkmul_ind8, f2, (x[c] = f2{threadIdx.x * 1e-3f + c + 1, 2.f + c}), x[c] = x[c] * (f2{a, a}), 8)
KERNEL(pkadd_dep, f2, (x[c] = f2{threadIdx.x * 1e-3f + c, 1.f + c}), x[c] = x[c] + (f2{b, b}), 1)
KERNEL(rsq_dep, S1, x[c].v = threadIdx.x * 1e-3f + c + 1, x[c].v = __builtin_amdgcn_rsqf(x[c].v), 1)
KERNEL(rsq_ind8, S1, x[c].v = threadIdx.x * 1e-3f + c + 1, x[c].v = __builtin_amdgcn_rsqf(x[c].v), 8)
KERNEL(rcp_dep, S1, x[c].v = threadIdx.x * 1e-3f + c + 1, x[c].v = __builtin_amdgcn_rcpf(x[c].v), 1)
KERNEL(rsqmul_dep, S1, x[c].v = threadIdx.x * 1e-3f + c + 1, x[c].v = __builtin_amdgcn_rsqf(x[c].v) * a, 1)
KERNEL(min3_dep, S1, x[c].v = threadIdx.x * 1e-3f + c + 1, x[c].v = fminf(fminf(x[c].v, a), b + x[c].v), 1)

template <typename K>
void run(const char* name, K k, int ops_per_iter_per_chain, int chains, float* out, long long* cyc) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, 1.0000001f, 1e-7f);
    hipDeviceSynchronize();
    long long best = 1LL << 62;
    for (int r = 0; r < 5; ++r) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, 1.0000001f, 1e-7f);
        long long c = 0;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        if (c < best) best = c;
    }
    const double instr = (double)N * ops_per_iter_per_chain * chains;
    printf("%-12s %7.2f cycles per wave-instruction (one wave alone)\n", name, best / instr);
}

int main() {
    float* out; long long* cyc;
    hipMalloc(&out, 64 * 4); hipMalloc(&cyc, 8);
    run("fma_dep", fma_dep, 1, 1, out, cyc);
    run("fma_ind8", fma_ind8, 1, 8, out, cyc);
    run("mul_dep", mul_dep, 1, 1, out, cyc);
    run("add_dep", add_dep, 1, 1, out, cyc);
    run("pkfma_dep", pkfma_dep, 1, 1, out, cyc);
    run("pkfma_ind8", pkfma_ind8, 1, 8, out, cyc);
    run("pkmul_dep", pkmul_dep, 1, 1, out, cyc);
    run("pkmul_ind8", pkmul_ind8, 1, 8, out, cyc);
    run("pkadd_dep", pkadd_dep, 1, 1, out, cyc);
    run("rsq_dep", rsq_dep, 1, 1, out, cyc);
    run("rsq_ind8", rsq_ind8, 1, 8, out, cyc);
    run("rcp_dep", rcp_dep, 1, 1, out, cyc);
    run("rsqmul_dep", rsqmul_dep, 2, 1, out, cyc);
    run("min3_dep", min3_dep, 2, 1, out, cyc);
    return 0;
}
