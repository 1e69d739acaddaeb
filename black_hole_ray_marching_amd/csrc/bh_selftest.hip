// bh_selftest.hip — on-device verification of the correctly rounded cores of bh_crmath.hpp against
// hipcc's IEEE division / sqrt (this TU: -ffp-contract=off, correctly rounded f32 div/sqrt).
// Exposed as bh_selftest_crmath (diagnostics API of include/bh_render.h).
#include "bh_common.hpp"
#include "bh_crmath.hpp"
#include "bh_srgb.hpp"

namespace bh {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// float with a uniformly random exponent in [elo, ehi] (unbiased exponents) and random mantissa/sign
__device__ __forceinline__ float rnd_float(uint64_t h, int elo, int ehi) {
    const uint32_t span = (uint32_t)(ehi - elo + 1);
    const uint32_t e = (uint32_t)(elo + 127) + (uint32_t)((h >> 32) % span);
    const uint32_t bits = ((uint32_t)(h >> 8) & 0x807FFFFFu) | (e << 23);
    return __uint_as_float(bits);
}

__device__ __forceinline__ void record(unsigned long long* cnt, uint32_t* ex, uint32_t a, uint32_t b, uint32_t got,
                                       uint32_t want) {
    const unsigned long long k = atomicAdd(cnt, 1ull);
    if (k < 2) { ex[4 * k + 0] = a; ex[4 * k + 1] = b; ex[4 * k + 2] = got; ex[4 * k + 3] = want; }
}

// op 0: sqrt_core over EVERY float with bits in [base, base + count) (guard-passing inputs only)
// op 1: div6 over every 32-bit pattern in [base, base + count) whose magnitude passes the key guard
// op 2: div_core on `count` random (n, d) pairs from the guarded domain, seeded by base
// op 3: div_core with n = d * m for random small integers m (exact quotients) and n = d*q +- ulps
// op 4: srgb_encode over every 32-bit pattern in [base, base + count) against a binary search of T
// op 6: srgb_encode_lut (table form) against srgb_encode over every 32-bit pattern in [base, base + count)
// op 10: srgb_encode_code (code-table form) against srgb_encode over every 32-bit pattern in [base, base + count)
// op 5: div12 over every 32-bit pattern in [base, base + count) whose magnitude passes the key guard
// op 8: atan2_core (+ its library fallback where flagged) against (float)atan2((double)y, (double)x) on
//       `count` random (y, x) pairs seeded by base: random directions, random magnitudes, and the
//       special values (+-0, axes, diagonals, tiny); ex[0..3] of a mismatch = y, x, got, want
// op 9: the unit-vector pairs of op 8 (10 of every 16); counts how many the core hands to the fallback
// op 11: wave_max_u32 (DPP scan) against a serial max, `count` rounds per wave
// op 12: rcp_from_rsq over EVERY q with bits in [base, base + count) whose Q = RN(RN(q*q) * sqrt_core(q))
//        passes the division guard, against the IEEE reciprocal 1/Q (ex = q, Q, got, want)
// op 13: for every q with bits in [base, base + count) whose rcp_from_rsq reciprocal r differs from RN(1/Q)
//        (op 12's mismatches: 1/Q within ~2^-41 of a rounding midpoint, r its faithful neighbour), div_core
//        with that r over EVERY numerator significand n in [1, 2) against the IEEE quotient n / Q; the
//        wave takes each such q in turn, its 64 lanes splitting the 2^23 numerators (ex = n, Q, got, want)
// op 7: div_core over EVERY pair of significands (n, d) in [1, 2)^2 with d's 23 fraction bits in
//       [base, base + count / 2^23): all 2^23 numerators per denominator (the full 2^46 square is
//       tools/ubench/cr_forms.hip; the tests cover blocks that include the extreme fractions)
__global__ void __launch_bounds__(256) selftest_kernel(int op, uint64_t base, uint64_t count,
                                                      unsigned long long* cnt, uint32_t* ex, const float* T,
                                                      const uint8_t* B, const uint32_t* E) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    if (op == 11) {
        // wave_max_u32 (bh_common.hpp, the DPP row scan of the tile costs) against a serial max over
        // the wave's lanes read one by one: `count` rounds of random values per wave (full waves: the
        // block is 256 threads), seeded by base; magnitudes from 0 to 2^32 - 1, often shared maxima
        const uint32_t lane = threadIdx.x & 63u;
        const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        for (uint64_t r = 0; r < count; ++r) {
            const uint64_t h = mix64((base + r) * 0x9E3779B97F4A7C15ull ^ ((w << 6) | lane));
            uint32_t v = (uint32_t)h >> ((h >> 32) & 31u);
            if (((h >> 40) & 7u) == 0u) v &= 0xFFu;
            const uint32_t got = wave_max_u32(v);
            uint32_t want = 0;
            for (int l = 0; l < 64; ++l) want = max(want, (uint32_t)__builtin_amdgcn_readlane((int)v, l));
            if (lane == 0u && got != want) record(cnt, ex, (uint32_t)w, (uint32_t)r, got, want);
        }
        return;
    }
    if (op == 13) {
        // wave-uniform trip count (every lane runs the same iterations; lanes past `count` test nothing)
        const uint32_t lane = threadIdx.x & 63u;
        const uint64_t w0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
        for (uint64_t b = w0; b < count; b += stride) {
            const uint64_t i = b + lane;
            bool bad = false;
            float Q = 0.0f, r = 0.0f;
            if (i < count) {
                const float q = __uint_as_float((uint32_t)(base + i));
                if (!crm::sqrt_bad(q)) {
                    const crm::SqrtY sy = crm::sqrt_core_y(q);
                    Q = (q * q) * sy.s;
                    if (!crm::div_d_bad(Q)) {
                        r = crm::rcp_from_rsq(Q, sy.y).r;
                        bad = __float_as_uint(r) != __float_as_uint(1.0f / Q);
                    }
                }
            }
            uint64_t m = __builtin_amdgcn_ballot_w64(bad);
            while (m) {
                const int l = __builtin_ctzll(m);
                m &= m - 1;
                const float Qw = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(Q), l));
                const float rw = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(r), l));
                for (uint32_t k = lane; k < (1u << 23); k += 64u) {
                    const float n = __uint_as_float(0x3F800000u | k);
                    const float got = crm::div_core(n, crm::Rcp{Qw, rw}), want = n / Qw;
                    if (__float_as_uint(got) != __float_as_uint(want))
                        record(cnt, ex, __float_as_uint(n), __float_as_uint(Qw), __float_as_uint(got), __float_as_uint(want));
                }
            }
        }
        return;
    }
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        if (op == 0) {
            const uint32_t bits = (uint32_t)(base + i);
            const float x = __uint_as_float(bits);
            if (crm::sqrt_bad(x)) continue;
            const float got = crm::sqrt_core(x), want = __builtin_sqrtf(x);
            if (__float_as_uint(got) != __float_as_uint(want) && !(got != got && want != want))
                record(cnt, ex, bits, 0, __float_as_uint(got), __float_as_uint(want));
        } else if (op == 1) {
            const uint32_t bits = (uint32_t)(base + i);
            const float x = __uint_as_float(bits);
            if (crm::key(x) < crm::KEY_MIN) continue;
            if (x != x || __builtin_isinf(x)) continue;
            const float got = crm::div6(x), want = x / 6.0f;
            if (__float_as_uint(got) != __float_as_uint(want))
                record(cnt, ex, bits, 0, __float_as_uint(got), __float_as_uint(want));
        } else if (op == 5) {
            const uint32_t bits = (uint32_t)(base + i);
            const float x = __uint_as_float(bits);
            if (crm::key(x) < crm::KEY_MIN) continue;
            if (x != x || __builtin_isinf(x)) continue;
            const float got = crm::div12(x), want = x / 12.0f;
            if (__float_as_uint(got) != __float_as_uint(want))
                record(cnt, ex, bits, 0, __float_as_uint(got), __float_as_uint(want));
        } else if (op == 6) {
            const uint32_t bits = (uint32_t)(base + i);
            const float x = __uint_as_float(bits);
            const uint32_t got = srgb_encode_lut(x, B, T), want = srgb_encode(x, T);  // op 4 pins srgb_encode
            if (got != want) record(cnt, ex, bits, 0, got, want);
        } else if (op == 10) {
            const uint32_t bits = (uint32_t)(base + i);
            const float x = __uint_as_float(bits);
            const uint32_t got = srgb_encode_code(x, E), want = srgb_encode(x, T);  // op 4 pins srgb_encode
            if (got != want) record(cnt, ex, bits, 0, got, want);
        } else if (op == 4) {
            const uint32_t bits = (uint32_t)(base + i);
            const float x = __uint_as_float(bits);
            const float xc = fminf(fmaxf(x, 0.0f), 1.0f);
            int lo = 0, hi = 256;  // largest k in [0, 255] with xc >= T[k]
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (xc >= T[mid]) lo = mid; else hi = mid;
            }
            const uint32_t got = srgb_encode(x, T);
            if (got != (uint32_t)lo) record(cnt, ex, bits, 0, got, (uint32_t)lo);
        } else if (op == 7) {
            const uint32_t dm = (uint32_t)(base + (i >> 23)) & 0x7FFFFFu, nm = (uint32_t)i & 0x7FFFFFu;
            const float d = __uint_as_float(0x3F800000u | dm), n = __uint_as_float(0x3F800000u | nm);
            const float got = crm::div_core(n, crm::rcp_refined(d)), want = n / d;
            if (__float_as_uint(got) != __float_as_uint(want))
                record(cnt, ex, __float_as_uint(n), __float_as_uint(d), __float_as_uint(got), __float_as_uint(want));
        } else if (op == 8 || op == 9) {
            const uint64_t h1 = mix64(base * 0x100000001B3ull + i), h2 = mix64(h1 ^ 0xD1B54A32D192ED03ull);
            float y, x;
            const uint32_t kind = (uint32_t)(h1 & 15u);
            if (kind < 10) {  // a unit vector's (z, x) as the shading sees them
                const float a = (float)((h2 >> 11) * 0x1p-53) * 6.283185307f, c = (float)((h1 >> 11) * 0x1p-53) * 2.0f - 1.0f;
                const float r = sqrtf(fmaxf(0.0f, 1.0f - c * c));
                y = r * sinf(a); x = r * cosf(a);
            } else if (kind < 13) {
                y = rnd_float(h1, -126, 10); x = rnd_float(h2, -126, 10);
                if (op == 9) continue;  // op 9: the rate over unit vectors only
            } else {
                if (op == 9) continue;
                const float sp[8] = {0.0f, -0.0f, 1.0f, -1.0f, 0x1p-130f, -0x1p-149f, 0.70710677f, 3.0f};
                y = sp[(h2 >> 3) & 7u]; x = sp[(h2 >> 6) & 7u];
                if ((h2 >> 9) & 1) x = y;       // diagonals
                if ((h2 >> 10) & 1) x = -x;
            }
            const crm::Atan2 at = crm::atan2_core(y, x);
            if (op == 9) {
                if (at.near) record(cnt, ex, __float_as_uint(y), __float_as_uint(x), __float_as_uint(at.f), 0u);
            } else {
                const float got = at.near ? (float)atan2((double)y, (double)x) : at.f;
                const float want = (float)atan2((double)y, (double)x);
                if (__float_as_uint(got) != __float_as_uint(want) && !(got != got && want != want))
                    record(cnt, ex, __float_as_uint(y), __float_as_uint(x), __float_as_uint(got), __float_as_uint(want));
            }
        } else if (op == 12) {
            const uint32_t bits = (uint32_t)(base + i);
            const float q = __uint_as_float(bits);
            if (crm::sqrt_bad(q)) continue;
            const crm::SqrtY sy = crm::sqrt_core_y(q);
            const float Q = (q * q) * sy.s;
            if (crm::div_d_bad(Q)) continue;
            const float got = crm::rcp_from_rsq(Q, sy.y).r, want = 1.0f / Q;
            if (__float_as_uint(got) != __float_as_uint(want))
                record(cnt, ex, bits, __float_as_uint(Q), __float_as_uint(got), __float_as_uint(want));
        } else if (op == 2 || op == 3) {
            const uint64_t h1 = mix64(base * 0x100000001B3ull + i), h2 = mix64(h1 ^ 0xD1B54A32D192ED03ull);
            float d = fabsf(rnd_float(h1, -40, 59));
            float n;
            if (op == 2) {
                n = rnd_float(h2, -60, 64);
                if ((h2 & 0xFF) == 7) n = ((h2 >> 9) & 1) ? -0.0f : 0.0f;
            } else {
                const float m = (float)((int32_t)((h2 >> 40) & 0xFFFF) - 32768);
                n = d * m;  // often exact
                const int32_t ulps = (int32_t)((h2 >> 8) & 7) - 3;
                n = __uint_as_float(__float_as_uint(n) + (uint32_t)ulps);
            }
            if (crm::div_d_bad(d) || crm::key(n) < crm::KEY_MIN || n != n || __builtin_isinf(n) || fabsf(n) > 0x1p64f) continue;
            const float got = crm::div_core(n, crm::rcp_refined(d)), want = n / d;
            if (__float_as_uint(got) != __float_as_uint(want))
                record(cnt, ex, __float_as_uint(n), __float_as_uint(d), __float_as_uint(got), __float_as_uint(want));
        }
    }
}

}  // namespace bh

extern "C" int bh_selftest_crmath(int op, uint64_t base, uint64_t count, uint64_t* out_mismatches,
                                  uint32_t* out_examples, int device) {
    if (op < 0 || op > 13 || !out_mismatches) return BH_ERR_INVALID_ARG;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) return BH_ERR_NO_DEVICE;
    unsigned long long* cnt = nullptr;
    uint32_t* ex = nullptr;
    float* T = nullptr;
    uint8_t* Bd = nullptr;
    uint32_t* Ed = nullptr;
    float table[bh::SRGB_TABLE];
    uint8_t btab[bh::SRGB_BUCKETS];
    uint32_t etab[bh::SRGB_CODES];
    (void)bh_srgb_encode_table(table);
    bh_srgb_bucket_table(table, btab);
    const bool etab_ok = bh_srgb_code_table(table, etab);
    int st = BH_OK;
    if (hipMalloc(&cnt, sizeof(*cnt)) != hipSuccess || hipMalloc(&ex, 8 * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&T, sizeof(table)) != hipSuccess || hipMalloc(&Bd, sizeof(btab)) != hipSuccess ||
        hipMalloc(&Ed, sizeof(etab)) != hipSuccess) {
        st = BH_ERR_OUT_OF_MEMORY;
    } else {
        (void)hipMemset(cnt, 0, sizeof(*cnt));
        (void)hipMemset(ex, 0, 8 * sizeof(uint32_t));
        (void)hipMemcpy(T, table, sizeof(table), hipMemcpyHostToDevice);
        (void)hipMemcpy(Bd, btab, sizeof(btab), hipMemcpyHostToDevice);
        (void)hipMemcpy(Ed, etab, sizeof(etab), hipMemcpyHostToDevice);
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
        hipLaunchKernelGGL(bh::selftest_kernel, dim3(cus * 8), dim3(256), 0, 0, op, base, count, cnt, ex, T, Bd, Ed);
        if (hipDeviceSynchronize() != hipSuccess) st = BH_ERR_HIP;
        unsigned long long h = 0;
        (void)hipMemcpy(&h, cnt, sizeof(h), hipMemcpyDeviceToHost);
        *out_mismatches = h + ((op == 10 && !etab_ok) ? 1u : 0u);
        if (out_examples) (void)hipMemcpy(out_examples, ex, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost);
    }
    if (cnt) (void)hipFree(cnt);
    if (ex) (void)hipFree(ex);
    if (T) (void)hipFree(T);
    if (Bd) (void)hipFree(Bd);
    if (Ed) (void)hipFree(Ed);
    (void)hipSetDevice(prev);
    return st;
}
