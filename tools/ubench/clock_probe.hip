// Shader clock probe (tools only): one wave spins for `spin` iterations and records the shader-clock
// counter (s_memtime) and the constant 100 MHz counter (s_memrealtime) at both ends, so
// MHz = 100 * d(memtime) / d(memrealtime).  Launched on a stream between frames, it reads the clock
// the GPU runs at right after each frame (tools/clock_series.py).
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/ubench/clock_probe.hip -o tools/ubench/clock_probe.so
#include <hip/hip_runtime.h>

__global__ void clock_probe_kernel(unsigned long long* out, int spin) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    float x = threadIdx.x * 1e-3f;
    for (int i = 0; i < spin; ++i) x = __builtin_fmaf(x, 0.999f, 1e-3f);
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = c1 - c0;
        out[1] = r1 - r0;
        out[2] = __float_as_uint(x);
    }
}

extern "C" int clock_probe(unsigned long long* out, int spin, hipStream_t s) {
    hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, s, out, spin);
    return (int)hipGetLastError();
}

// Memory latency probe: one lane chases `n` dependent pointers through `chain` (a random cycle over a
// buffer far larger than L2 + MALL), s_memrealtime around it: ns per dependent load.
__global__ void chase_kernel(const unsigned int* __restrict__ chain, unsigned long long* out, int n) {
    unsigned int p = 0;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < n; ++i) p = __builtin_nontemporal_load(&chain[p]);
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = r1 - r0;
        out[1] = p;
    }
}

extern "C" int chase_probe(const unsigned int* chain, unsigned long long* out, int n, hipStream_t s) {
    hipLaunchKernelGGL(chase_kernel, dim3(1), dim3(1), 0, s, chain, out, n);
    return (int)hipGetLastError();
}

// Whole-chip clock probe: `blocks` one-wave workgroups (dispatched round-robin over the XCDs), each
// timing the same FMA spin with s_memtime / s_memrealtime and recording its XCD (HW_REG_XCC_ID):
// out[b] = {d(memtime), d(memrealtime), xcc}.  Per-XCD shader clock = 100 MHz * dm / dr.
__global__ void chip_clock_kernel(unsigned long long* out, int spin) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    float x = threadIdx.x * 1e-3f;
    for (int i = 0; i < spin; ++i) x = __builtin_fmaf(x, 0.999f, 1e-3f);
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    const unsigned int xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;  // HW_REG_XCC_ID[3:0]
    if (threadIdx.x == 0) {
        out[4 * blockIdx.x + 0] = c1 - c0;
        out[4 * blockIdx.x + 1] = r1 - r0;
        out[4 * blockIdx.x + 2] = xcc;
        out[4 * blockIdx.x + 3] = __float_as_uint(x);
    }
}

extern "C" int chip_clock_probe(unsigned long long* out, int blocks, int spin, hipStream_t s) {
    hipLaunchKernelGGL(chip_clock_kernel, dim3(blocks), dim3(64), 0, s, out, spin);
    return (int)hipGetLastError();
}

// Heavy-load clock probe: `blocks` x 256 threads (all waves resident at 8 per SIMD when blocks = 8 x
// CUs), each lane running 8 independent FMA chains for `spin` iterations -- VALU-bound like a frame.
// out[b] = {d(memtime), d(memrealtime), xcc} of each block's first wave.
__global__ void __launch_bounds__(256) heavy_clock_kernel(unsigned long long* out, int spin) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    float x[8];
    for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < spin; ++i) {
#pragma unroll
        for (int c = 0; c < 8; ++c) x[c] = __builtin_fmaf(x[c], 0.999f, 1e-3f);
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    const unsigned int xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
    float s = 0.0f;
    for (int c = 0; c < 8; ++c) s += x[c];
    if (threadIdx.x == 0) {
        out[4 * blockIdx.x + 0] = c1 - c0;
        out[4 * blockIdx.x + 1] = r1 - r0;
        out[4 * blockIdx.x + 2] = xcc;
        out[4 * blockIdx.x + 3] = __float_as_uint(s);
    }
}

extern "C" int heavy_clock_probe(unsigned long long* out, int blocks, int spin, hipStream_t s) {
    hipLaunchKernelGGL(heavy_clock_kernel, dim3(blocks), dim3(256), 0, s, out, spin);
    return (int)hipGetLastError();
}
