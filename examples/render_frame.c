/*
 * render_frame.c -- the C ABI on its own: what a non-Python host (the reference's Rust crate through
 * `extern "C"`) does with libbh_render.so.  Plain C, no torch: the HIP runtime's C API
 * allocates the caller-owned device targets, the ABI does the rest.
 *
 *   Scene::new  -> bh_synthetic_sky + bh_create + bh_camera_default + bh_camera_uniform_update + bh_uniforms_default
 *   Scene::render -> bh_render (RGBA32F col + blackout_col, exact math)
 *
 * Renders one W x H frame, copies both targets back, prints a checksum line (FNV-1a over the bytes of
 * each target, per-fate pixel counts) and optionally writes the colour target as a binary PPM.
 *   examples/render_frame [W H cap out.ppm]
 * Built by black_hole_ray_marching_amd/build.py (gcc, C11); run by tests/test_gpu_c_example.py.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "bh_render.h"

#define CHECK_BH(x)                                                                          \
    do {                                                                                     \
        int s_ = (x);                                                                        \
        if (s_ != BH_OK) {                                                                   \
            fprintf(stderr, "%s: %s (%s)\n", #x, bh_status_string(s_), bh_last_error());      \
            return 2;                                                                        \
        }                                                                                    \
    } while (0)
#define CHECK_HIP(x)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                          \
            return 3;                                                                        \
        }                                                                                    \
    } while (0)

static uint64_t fnv1a(const uint8_t* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

int main(int argc, char** argv) {
    const uint32_t W = argc > 2 ? (uint32_t)atoi(argv[1]) : 512, H = argc > 2 ? (uint32_t)atoi(argv[2]) : 256;
    const uint32_t cap = argc > 3 ? (uint32_t)atoi(argv[3]) : 512;
    const char* ppm = argc > 4 ? argv[4] : NULL;
    if (bh_abi_version() != BH_ABI_VERSION) {
        fprintf(stderr, "ABI version %d, header %d\n", bh_abi_version(), BH_ABI_VERSION);
        return 1;
    }
    const uint32_t sw = 1024, sh = 512;
    uint8_t* sky = (uint8_t*)malloc((size_t)sw * sh * 4);
    CHECK_BH(bh_synthetic_sky(sky, sw, sh, 0x5EEDB1AC401Eull));
    bh_ctx* ctx = NULL;
    CHECK_BH(bh_create(sky, sw, sh, 0, &ctx));
    bh_camera cam;
    bh_camera_uniform cu;
    bh_uniforms u;
    CHECK_BH(bh_camera_default(W, H, &cam));
    CHECK_BH(bh_camera_uniform_update(&cam, &cu));
    CHECK_BH(bh_uniforms_default(&u));

    const size_t px = (size_t)W * H, bytes = px * 16;
    void *d_col = NULL, *d_bo = NULL;
    uint8_t* d_fate = NULL;
    CHECK_HIP(hipMalloc(&d_col, bytes));
    CHECK_HIP(hipMalloc(&d_bo, bytes));
    CHECK_HIP(hipMalloc((void**)&d_fate, px));
    bh_render_desc d = {0};
    d.width = W; d.height = H; d.max_iters = cap; d.scene_flags = BH_SCENE_DEFAULT;
    d.format = BH_OUT_RGBA32F; d.math = BH_MATH_EXACT; d.layout = BH_LAYOUT_ROWMAJOR;
    d.shard_index = 0; d.shard_count = 1; d.schedule = BH_SCHED_TILE;
    d.out_col = d_col; d.out_blackout = d_bo; d.dbg_fate = d_fate;
    CHECK_BH(bh_render(ctx, &cu, &u, &d, NULL));  /* NULL stream: the legacy default stream */
    CHECK_HIP(hipDeviceSynchronize());

    float* col = (float*)malloc(bytes);
    float* bo = (float*)malloc(bytes);
    uint8_t* fate = (uint8_t*)malloc(px);
    CHECK_HIP(hipMemcpy(col, d_col, bytes, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(bo, d_bo, bytes, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(fate, d_fate, px, hipMemcpyDeviceToHost));
    size_t nf[4] = {0, 0, 0, 0};
    for (size_t i = 0; i < px; ++i) nf[fate[i] & 3u]++;
    printf("{\"width\": %u, \"height\": %u, \"max_iters\": %u, \"col_fnv1a\": \"%016llx\", \"blackout_fnv1a\": \"%016llx\", "
           "\"fates\": {\"cap\": %zu, \"escape\": %zu, \"surface\": %zu, \"blackout\": %zu}}\n",
           W, H, cap, (unsigned long long)fnv1a((const uint8_t*)col, bytes),
           (unsigned long long)fnv1a((const uint8_t*)bo, bytes), nf[0], nf[1], nf[2], nf[3]);
    if (ppm) {
        FILE* f = fopen(ppm, "wb");
        if (!f) return 4;
        fprintf(f, "P6\n%u %u\n255\n", W, H);
        for (size_t i = 0; i < px; ++i)
            for (int c = 0; c < 3; ++c) {
                float v = col[4 * i + c];
                v = v != v ? 0.0f : (v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v));
                fputc((int)lrintf(v * 255.0f), f);
            }
        fclose(f);
    }
    (void)hipFree(d_col);
    (void)hipFree(d_bo);
    (void)hipFree(d_fate);
    CHECK_BH(bh_destroy(ctx));
    free(sky); free(col); free(bo); free(fate);
    return 0;
}
