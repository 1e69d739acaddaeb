// raw_ops.hip — how far are gfx950's raw v_sqrt_f32 / v_rcp_f32 from the correctly rounded results?
// Counts mismatches over EVERY positive normal float (and the subnormals separately).
//   hipcc --offload-arch=gfx950 -O3 -fhip-fp32-correctly-rounded-divide-sqrt tools/ubench/raw_ops.hip -o /tmp/raw_ops
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(uint32_t lo, uint32_t hi, unsigned long long* cnt, uint32_t* ex) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; lo + i < hi; i += stride) {
        const uint32_t b = lo + (uint32_t)i;
        const float x = __uint_as_float(b);
        const float s_raw = __builtin_amdgcn_sqrtf(x), s_ok = __builtin_sqrtf(x);
        const float r_raw = __builtin_amdgcn_rcpf(x), r_ok = 1.0f / x;
        const float q_raw = __builtin_amdgcn_rsqf(x);
        if (__float_as_uint(s_raw) != __float_as_uint(s_ok)) {
            const unsigned long long k = atomicAdd(&cnt[0], 1ull);
            if (k < 4) ex[k] = b;
        }
        if (__float_as_uint(r_raw) != __float_as_uint(r_ok)) atomicAdd(&cnt[1], 1ull);
        // rsq vs RN(1/RN(sqrt)) is not a CR reference; report |ulp diff| > 1 only as a sanity check
        const float q_ref = 1.0f / s_ok;
        const int d = (int)__float_as_uint(q_raw) - (int)__float_as_uint(q_ref);
        if (d > 1 || d < -1) atomicAdd(&cnt[2], 1ull);
    }
}

int main() {
    unsigned long long* cnt; uint32_t* ex;
    hipMalloc(&cnt, 4 * sizeof(unsigned long long)); hipMalloc(&ex, 16);
    struct { const char* name; uint32_t lo, hi; } R[] = {{"normal", 0x00800000u, 0x7F800000u},
                                                         {"subnormal", 0x00000001u, 0x00800000u}};
    for (auto& r : R) {
        hipMemset(cnt, 0, 4 * sizeof(unsigned long long)); hipMemset(ex, 0, 16);
        probe<<<4096, 256>>>(r.lo, r.hi, cnt, ex);
        unsigned long long h[4]; uint32_t e[4];
        hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost); hipMemcpy(e, ex, sizeof e, hipMemcpyDeviceToHost);
        printf("%-9s inputs %u: raw v_sqrt != CR sqrt: %llu   raw v_rcp != CR 1/x: %llu   |rsq - 1/sqrt| > 1ulp: %llu\n",
               r.name, r.hi - r.lo, h[0], h[1], h[2]);
        for (int k = 0; k < 4 && k < (int)h[0]; ++k) printf("  sqrt example: 0x%08x\n", e[k]);
    }
    return 0;
}
