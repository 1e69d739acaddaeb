/* bh_bloom_oracle.c — TEST INFRASTRUCTURE: CPU restatement of the reference's post-processing chain
 * (Kawase bloom + remix), the checker for the product's bh_bloom.  Never
 * linked into the product library.
 *
 * PARITY UNPINNED (as the march oracle, bh_oracle.c header): the reference (Rust + wgpu) cannot run
 * here and ships no fixtures.  This is a pass-by-pass restatement of
 *   src/bloom.rs:53-71 (Bloom::render, levels = 3 from src/state.rs:125),
 *   src/blur.rs:37-45 (Blur::render = downsampling then upsampling),
 *   src/kawase_downsampling.rs:30-39 (resolutions), :250-306 (render), bind groups :181-225,
 *   src/kawase_upsampling.rs:32-39 (resolutions), :192-210 (bind group `level` = texture
 *     [levels-level-1] with resolution uniform [level]), :241-295 (render),
 *   src/kawase_downsample.wgsl:23-36 (returns the centre tap only), src/kawase_upsample.wgsl:23-38,
 *   src/remix.wgsl:20-25, src/copy.wgsl:15-19, src/screen_triangle.wgsl:16-24 (texcoord),
 * with every texture Bgra8UnormSrgb (src/copy.rs:132, src/remix.rs:160, src/kawase_*sampling.rs
 * create_textures): each pass decodes its inputs through the sRGB table and its output is stored
 * through the normative encode (bho_srgb_encode).
 *
 * Normative sampling (WGSL leaves the filter's precision to the implementation): a target pixel
 * (x, y) of a w x h pass has texcoord u = (x+0.5)/w, v = (y+0.5)/h in f32; textureSample /
 * textureSampleLevel at (u, v) of a tw x th texture is the clamp-to-edge bilinear filter with f32
 * weights of bh_oracle.c's sky sampler (tx = u*tw - 0.5, lerp along x then y), on decoded texels;
 * every sampler of the chain filters linearly at the scales it is used (mag = min = Linear for the
 * copy/Kawase samplers; remix's min = Nearest never applies: its inputs are sampled 1:1, LOD 0).
 * Alpha: linear unorm (a/255), stored round-half-up; every texel of the chain has alpha 1.
 * Texture rows are tightly packed BGRA8 (byte 0 = B).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

void bho_srgb_lut(float lut[256]);
uint8_t bho_srgb_encode(float x);

typedef struct { uint32_t w, h; uint8_t* px; } tex_t;   /* BGRA8 */
typedef struct { float c[4]; } rgba;                     /* r, g, b, a (linear) */

static float g_lut[256];

static tex_t tex_new(uint32_t w, uint32_t h) {
    tex_t t = {w, h, (uint8_t*)calloc((size_t)w * h, 4)};
    return t;
}
static void tex_free(tex_t* t) { free(t->px); t->px = NULL; }

static rgba texel(const tex_t* t, int32_t x, int32_t y) {
    const uint8_t* p = t->px + ((size_t)y * t->w + (size_t)x) * 4u;
    rgba r = {{g_lut[p[2]], g_lut[p[1]], g_lut[p[0]], (float)p[3] / 255.0f}};
    return r;
}
static int32_t clampi(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* clamp-to-edge bilinear of decoded texels at texcoord (u, v) */
static rgba sample(const tex_t* t, float u, float v) {
    float tx = u * (float)t->w - 0.5f, ty = v * (float)t->h - 0.5f;
    tx = fminf(fmaxf(tx, -1.0f), (float)t->w);
    ty = fminf(fmaxf(ty, -1.0f), (float)t->h);
    const float fx0 = floorf(tx), fy0 = floorf(ty);
    const float fa = tx - fx0, fb = ty - fy0;
    const int32_t wm = (int32_t)t->w - 1, hm = (int32_t)t->h - 1;
    int32_t x0 = (int32_t)fx0, y0 = (int32_t)fy0;
    const int32_t x1 = clampi(x0 + 1, 0, wm), y1 = clampi(y0 + 1, 0, hm);
    x0 = clampi(x0, 0, wm);
    y0 = clampi(y0, 0, hm);
    const rgba t00 = texel(t, x0, y0), t10 = texel(t, x1, y0), t01 = texel(t, x0, y1), t11 = texel(t, x1, y1);
    const float ia = 1.0f - fa, ib = 1.0f - fb;
    rgba r;
    for (int k = 0; k < 4; k++) {
        const float top = t00.c[k] * ia + t10.c[k] * fa;
        const float bot = t01.c[k] * ia + t11.c[k] * fa;
        r.c[k] = top * ib + bot * fb;
    }
    return r;
}

static uint8_t unorm8(float a) {
    if (!(a > 0.0f)) return 0;
    if (a >= 1.0f) return 255;
    return (uint8_t)floor((double)a * 255.0 + 0.5);
}
static void store(tex_t* t, uint32_t x, uint32_t y, rgba c) {
    uint8_t* p = t->px + ((size_t)y * t->w + x) * 4u;
    p[0] = bho_srgb_encode(c.c[2]);
    p[1] = bho_srgb_encode(c.c[1]);
    p[2] = bho_srgb_encode(c.c[0]);
    p[3] = unorm8(c.c[3]);
}

typedef enum { SH_COPY, SH_DOWN, SH_UP, SH_REMIX } shader_t;

/* one full-screen pass into `out`: shader over inputs a (and b for remix), resolution uniform res */
static void pass(shader_t sh, const tex_t* a, const tex_t* b, const uint32_t res[2], tex_t* out) {
#pragma omp parallel for schedule(static)
    for (long long yy = 0; yy < (long long)out->h; yy++) {
        const uint32_t y = (uint32_t)yy;
        for (uint32_t x = 0; x < out->w; x++) {
            const float u = ((float)x + 0.5f) / (float)out->w;   /* screen_triangle texcoord */
            const float v = ((float)y + 0.5f) / (float)out->h;
            rgba c;
            if (sh == SH_COPY || sh == SH_DOWN) {
                /* copy.wgsl:17; kawase_downsample.wgsl:35 returns textureSample(uv) (the 4 taps
                 * summed at :30-33 are unused) */
                c = sample(a, u, v);
            } else if (sh == SH_UP) {
                /* kawase_upsample.wgsl:25-38 */
                const float hx = 0.5f / (float)res[0], hy = 0.5f / (float)res[1];
                const float o = 3.0f;
                const float du[8] = {(-hx * 2.0f) * o, (-hx) * o, 0.0f * o, hx * o, (hx * 2.0f) * o, hx * o, 0.0f * o, (-hx) * o};
                const float dv[8] = {0.0f * o, hy * o, (hy * 2.0f) * o, hy * o, 0.0f * o, (-hy) * o, (-hy * 2.0f) * o, (-hy) * o};
                rgba s = sample(a, u + du[0], v + dv[0]);
                for (int i = 1; i < 8; i++) {
                    const rgba t = sample(a, u + du[i], v + dv[i]);
                    const float wgt = (i & 1) ? 2.0f : 1.0f;
                    for (int k = 0; k < 4; k++) s.c[k] = s.c[k] + ((i & 1) ? t.c[k] * wgt : t.c[k]);
                }
                for (int k = 0; k < 4; k++) c.c[k] = s.c[k] / 12.0f;
            } else {
                /* remix.wgsl:22-24: col_0 + col_1 * 0.5 */
                const rgba c0 = sample(a, u, v), c1 = sample(b, u, v);
                for (int k = 0; k < 4; k++) c.c[k] = c0.c[k] + c1.c[k] * 0.5f;
            }
            store(out, x, y, c);
        }
    }
}

/* Blur::render (blur.rs:37-45) of `input` (its downsampling.textures[0]) into `out`. */
static void blur(const tex_t* input, uint32_t W, uint32_t H, uint32_t levels, tex_t* out) {
    uint32_t res[16][2];
    uint32_t w = W, h = H;
    for (uint32_t l = 0; l < levels; l++) {              /* kawase_*sampling.rs resolutions */
        w = w ? w : 1; h = h ? h : 1;
        res[l][0] = w; res[l][1] = h;
        w /= 2; h /= 2;
    }
    tex_t down[16], up[16];
    for (uint32_t l = 0; l < levels; l++) {
        down[l] = tex_new(res[l][0], res[l][1]);
        up[l] = tex_new(res[l][0], res[l][1]);
    }
    memcpy(down[0].px, input->px, (size_t)W * H * 4u);  /* the copy pass wrote down[0] (Bloom::render) */
    /* KawaseDownsampling::render: passes 1..levels-1 write textures[l] with bind group l-1, then
     * the final pass writes upsampling.textures[levels-1] (its input) with bind group levels-1 */
    for (uint32_t l = 1; l < levels; l++) pass(SH_DOWN, &down[l - 1], NULL, res[l - 1], &down[l]);
    pass(SH_DOWN, &down[levels - 1], NULL, res[levels - 1], &up[levels - 1]);
    /* KawaseUpsampling::render: pass `l` (0..levels-2) writes textures[levels-l-2] with bind group
     * l = (textures[levels-l-1], resolution[l]); the final pass writes `out` with bind group
     * levels-1 = (textures[0], resolution[levels-1]) */
    for (uint32_t l = 0; l + 1 < levels; l++) pass(SH_UP, &up[levels - l - 1], NULL, res[l], &up[levels - l - 2]);
    pass(SH_UP, &up[0], NULL, res[levels - 1], out);
    for (uint32_t l = 0; l < levels; l++) { tex_free(&down[l]); tex_free(&up[l]); }
}

/* Bloom::render (bloom.rs:53-71) with `levels` blurs: col / blackout are the scene's two targets
 * (full_image_input = final_remix input 0, blackout_input = copies[0] input), out = the surface. */
int bho_bloom(const uint8_t* col, const uint8_t* blackout, uint32_t W, uint32_t H, uint32_t levels,
              uint8_t* out, int threads) {
    if (!col || !blackout || !out || W == 0 || H == 0 || levels < 1 || levels > 16) return -1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
    bho_srgb_lut(g_lut);
    const uint32_t full[2] = {W, H};
    const size_t bytes = (size_t)W * H * 4u;
    tex_t copy_in[16], remix_in0[16], remix_in1[16], blur_in, final_in0, final_in1, surf;
    for (uint32_t l = 0; l < levels; l++) {
        copy_in[l] = tex_new(W, H); remix_in0[l] = tex_new(W, H); remix_in1[l] = tex_new(W, H);
    }
    blur_in = tex_new(W, H); final_in0 = tex_new(W, H); final_in1 = tex_new(W, H);
    surf.w = W; surf.h = H; surf.px = out;
    memcpy(copy_in[0].px, blackout, bytes);
    memcpy(final_in0.px, col, bytes);
    /* the loop always uses copies[0], blurs[0], remixes[0] (bloom.rs:59-62) */
    for (uint32_t level = 0; level + 1 < levels; level++) {
        pass(SH_COPY, &copy_in[0], NULL, full, &blur_in);          /* copies[0] -> blurs[0].input */
        pass(SH_COPY, &copy_in[0], NULL, full, &remix_in0[0]);     /* copies[0] -> remixes[0].input_0 */
        blur(&blur_in, W, H, 1, &remix_in1[0]);                    /* blurs[0] (1 level) */
        pass(SH_REMIX, &remix_in0[0], &remix_in1[0], full, &copy_in[level + 1]);
    }
    const uint32_t L = levels - 1;
    pass(SH_COPY, &copy_in[L], NULL, full, &blur_in);
    pass(SH_COPY, &copy_in[L], NULL, full, &remix_in0[L]);
    blur(&blur_in, W, H, levels, &remix_in1[L]);                   /* blurs[levels-1] (levels levels) */
    pass(SH_REMIX, &remix_in0[L], &remix_in1[L], full, &final_in1);
    pass(SH_REMIX, &final_in0, &final_in1, full, &surf);           /* final_remix -> output */
    for (uint32_t l = 0; l < levels; l++) { tex_free(&copy_in[l]); tex_free(&remix_in0[l]); tex_free(&remix_in1[l]); }
    tex_free(&blur_in); tex_free(&final_in0); tex_free(&final_in1);
    return 0;
}
