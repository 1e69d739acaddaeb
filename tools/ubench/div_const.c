/* Host-side exhaustive check of crm::div6 / crm::div12 (bh_crmath.hpp): x/D as fma(x, H, x*L) with
 * H = RD_f32(1/D), L = RN_f32(1/D - H), against the IEEE quotient x/D, over every finite float
 * (x86 FMA, correctly rounded like v_fma_f32).  Reports mismatches inside the callers' domain
 * (x == 0 or |x| >= 2^-60) and the largest mismatching |x| overall.
 *   gcc -O2 -mfma -fopenmp -ffp-contract=off tools/ubench/div_const.c -o /tmp/div_const -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static float fb(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }
static uint32_t bf(float f) { uint32_t b; memcpy(&b, &f, 4); return b; }
int main(void) {
    int rc = 0;
    for (int D = 6; D <= 12; D += 6) {
        const double inv = 1.0 / D;
        float H = (float)inv;
        if ((double)H > inv) H = nextafterf(H, 0.0f);
        const float L = (float)(inv - (double)H);
        unsigned long long bad = 0, n = 0;
        uint32_t worst = 0;
#pragma omp parallel for reduction(+ : bad, n) reduction(max : worst) schedule(static)
        for (long long i = 0; i < 0x7f800000LL; ++i) {
            for (int sg = 0; sg < 2; ++sg) {
                const uint32_t b = (uint32_t)i | (sg ? 0x80000000u : 0u);
                const float x = fb(b);
                if (bf(fmaf(x, H, x * L)) == bf(x / (float)D)) continue;
                if ((uint32_t)i > worst) worst = (uint32_t)i;
                if (x == 0.0f || fabsf(x) >= 0x1p-60f) ++bad;
            }
            ++n;
        }
        printf("D=%d H=%a L=%a: %llu magnitudes, %llu mismatches in the domain, largest mismatching |x| %a\n",
               D, H, L, n, bad, fb(worst));
        rc |= bad != 0;
    }
    return rc;
}
