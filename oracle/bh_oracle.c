/*
 * bh_oracle.c — CPU ORACLE for the geodesic ray-march hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / the timed CPU baseline.  The product (libbh_render.so) never links it.
 *
 * PARITY UNPINNED: the reference (Rust + WGSL, wgpu 22.1) cannot be compiled or run in this
 * environment (no cargo/rustc, no WGSL compiler, no GPU in the build container) and it ships no
 * tests, golden vectors or fixtures.  This file is therefore a line-by-line
 * restatement of src/black_hole_maybe.wgsl, cross-checked against an independent numpy
 * restatement (oracle/oracle_np.py) and physics known-answer tests (tests/test_oracle_kat.py).
 *
 * Where WGSL leaves precision implementation-defined, this restatement fixes one normative choice
 * (DESIGN.md "Normative arithmetic"):
 *   - f32 + - * / sqrt are IEEE-754 correctly rounded, evaluated in WGSL source order, no FMA
 *     contraction (build with -ffp-contract=off, no -ffast-math);
 *   - length(v) = sqrt(dot(v,v)), dot = (x*x + y*y) + z*z, normalize(v) = v / length(v);
 *   - pow(q, 2.5) = (q * q) * sqrt(q)   (f32, three correctly rounded ops; <= 1.5 ulp of q^2.5);
 *   - pow(c, 1.5) = c * sqrt(c)         (f32);
 *   - atan2(y, x) = (float)atan2((double)y, (double)x);
 *   - textureSampleLevel on Rgba8UnormSrgb with a mag=Linear, clamp-to-edge sampler = decode each
 *     texel through the 256-entry sRGB->linear table, then bilinear with fp32 weights
 *     (lerp along u, then along v); a NaN coordinate samples texel (0,0).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/bh_render.h"

#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 smul(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }
static inline v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 divs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
static inline float dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline float len(v3 a) { return sqrtf(dot(a, a)); }
static inline v3 normalize(v3 a) { return divs(a, len(a)); }
static inline v3 cross(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float pow25(float q) { return (q * q) * sqrtf(q); }
static inline float pow15(float c) { return c * sqrtf(c); }

/* Parity-envelope variants (bho_render_rows_variant; DESIGN.md §3 "Parity envelope"): choices a real
 * WGSL implementation may make where WGSL leaves precision to the implementation, instead of the
 * normative ones above.  0 = normative (what every parity test uses). */
#define BHO_V_POW_EXP2LOG2 1u /* pow(x, e) = exp2(e * log2(x)) in f32 (how GPU compilers lower pow) */
#define BHO_V_TEX_8BIT 2u     /* bilinear weights quantised to 8 fractional bits (texture units) */
#define BHO_V_TEX_NEAREST 4u  /* LOD 0 treated as minification: min_filter = Nearest (src/texture.rs:66-67) */
#define BHO_V_ATAN2F 8u       /* atan2 evaluated in f32 (libm atan2f) */
static inline float powv(float x, float e, uint32_t variant) {
    if (!(variant & BHO_V_POW_EXP2LOG2)) return e == 2.5f ? pow25(x) : pow15(x);
    return x > 0.0f ? exp2f(e * log2f(x)) : (x == 0.0f ? 0.0f : NAN);
}

/* constants, src/black_hole_maybe.wgsl:80-85 (abstract floats rounded to f32 at use) */
#define MIN_DIST 0.001f
#define TWO_PI 6.28318530718f
#define ONE_PI 3.14159265359f

typedef struct {
    float RS, DTM, MAX_DIST, DP;
    uint32_t BLACKOUT_EH;
    uint32_t flags;
    uint32_t max_iters;
    uint32_t variant;  /* BHO_V_* (0 = normative) */
} params;

/* sdf_sphere, :91-93 — length(centre - p) - r */
static inline float sdf_sphere(v3 p, v3 c, float r) { return len(sub(c, p)) - r; }
/* sdf_plane, :95-97 */
static inline float sdf_plane(v3 p, float y) { return fabsf(p.y - y) - 0.02f; }
/* sdf_cylinder, :99-101 — length(p.xz - pos) - radius */
static inline float sdf_cylinder(v3 p, float px, float pz, float radius) {
    float dx = p.x - px, dz = p.z - pz;
    return sqrtf(dx * dx + dz * dz) - radius;
}
/* sdf_accretion_disk, :103-105 */
static inline float sdf_accretion_disk(v3 p, v3 c, float big_r, float little_r) {
    float a = sdf_cylinder(p, c.x, c.z, big_r);
    float b = -sdf_cylinder(p, c.x, c.z, little_r);
    return fmaxf(fmaxf(a, b), sdf_plane(p, c.y));
}
/* sdf_markers, :107-117 */
static inline float sdf_markers(v3 p) {
    float s1 = sdf_sphere(p, mk(0.0f, 10.0f, -10.0f), 0.5f);
    float s2 = sdf_sphere(p, mk(0.0f, -10.0f, -10.0f), 0.5f);
    float s3 = sdf_sphere(p, mk(10.0f, 0.0f, -10.0f), 0.5f);
    float s4 = sdf_sphere(p, mk(-10.0f, 0.0f, -10.0f), 0.5f);
    return fminf(s1, fminf(s2, fminf(s3, s4)));
}
/* sdf, :119-123 (scene_flags select the terms; the reference always has both) */
static inline float sdf(const params* P, v3 p) {
    float d = INFINITY;
    if (P->flags & BH_SCENE_DISC) d = sdf_accretion_disk(p, mk(0.0f, 0.0f, 0.0f), 6.0f * P->RS, 3.0f * P->RS);
    if (P->flags & BH_SCENE_MARKERS) {
        float m = sdf_markers(p);
        d = (P->flags & BH_SCENE_DISC) ? fminf(d, m) : m;
    }
    return d;
}
/* rd_derivative, :125-127 — ((((DP * RS) * -1.5) * h2) * ro) / pow(dot(ro, ro), 2.5) */
static inline v3 rd_derivative(const params* P, v3 ro, float h2) {
    float s = ((P->DP * P->RS) * -1.5f) * h2;
    return divs(smul(s, ro), powv(dot(ro, ro), 2.5f, P->variant));
}
/* get_delta_photon_rk4, :134-151 */
static inline void rk4(const params* P, v3 ro, v3 rd, float dt, float h2, v3* dro, v3* drd) {
    v3 ro_k1 = smul(dt, rd);
    v3 rd_k1 = smul(dt, rd_derivative(P, ro, h2));
    v3 ro_k2 = smul(dt, add(rd, smul(0.5f, rd_k1)));
    v3 rd_k2 = smul(dt, rd_derivative(P, add(ro, smul(0.5f, ro_k1)), h2));
    v3 ro_k3 = smul(dt, add(rd, smul(0.5f, rd_k2)));
    v3 rd_k3 = smul(dt, rd_derivative(P, add(ro, smul(0.5f, ro_k2)), h2));
    v3 ro_k4 = smul(dt, add(rd, rd_k3));
    v3 rd_k4 = smul(dt, rd_derivative(P, add(ro, ro_k3), h2));
    *dro = divs(add(add(add(ro_k1, smul(2.0f, ro_k2)), smul(2.0f, ro_k3)), ro_k4), 6.0f);
    *drd = divs(add(add(add(rd_k1, smul(2.0f, rd_k2)), smul(2.0f, rd_k3)), rd_k4), 6.0f);
}

typedef struct {
    const uint8_t* tex;
    uint32_t w, h;
    float lut[256];
    uint32_t variant;  /* BHO_V_TEX_* */
} sky_t;

/* Rgba8UnormSrgb texel fetch + decode (src/texture.rs:41) */
static inline v3 texel(const sky_t* S, int32_t x, int32_t y) {
    const uint8_t* t = S->tex + ((size_t)y * S->w + (size_t)x) * 4u;
    return mk(S->lut[t[0]], S->lut[t[1]], S->lut[t[2]]);
}
static inline int32_t clampi(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* textureSampleLevel(t_diffuse, s_diffuse, uv, 0.0).xyz with the sampler of src/texture.rs:62-70 */
static v3 sample_bilinear(const sky_t* S, float u, float v) {
    if (u != u || v != v) return texel(S, 0, 0); /* Q8 */
    if (S->variant & BHO_V_TEX_NEAREST) {
        int32_t nx = (int32_t)floorf(fminf(fmaxf(u, 0.0f), 1.0f) * (float)S->w);
        int32_t ny = (int32_t)floorf(fminf(fmaxf(v, 0.0f), 1.0f) * (float)S->h);
        return texel(S, clampi(nx, 0, (int32_t)S->w - 1), clampi(ny, 0, (int32_t)S->h - 1));
    }
    float tx = u * (float)S->w - 0.5f;
    float ty = v * (float)S->h - 0.5f;
    tx = fminf(fmaxf(tx, -1.0f), (float)S->w);
    ty = fminf(fmaxf(ty, -1.0f), (float)S->h);
    float fx0 = floorf(tx), fy0 = floorf(ty);
    float a = tx - fx0, b = ty - fy0;
    if (S->variant & BHO_V_TEX_8BIT) { a = rintf(a * 256.0f) / 256.0f; b = rintf(b * 256.0f) / 256.0f; }
    int32_t x0 = (int32_t)fx0, y0 = (int32_t)fy0;
    int32_t x1 = clampi(x0 + 1, 0, (int32_t)S->w - 1), y1 = clampi(y0 + 1, 0, (int32_t)S->h - 1);
    x0 = clampi(x0, 0, (int32_t)S->w - 1);
    y0 = clampi(y0, 0, (int32_t)S->h - 1);
    v3 t00 = texel(S, x0, y0), t10 = texel(S, x1, y0), t01 = texel(S, x0, y1), t11 = texel(S, x1, y1);
    float ia = 1.0f - a, ib = 1.0f - b;
    v3 top = add(muls(t00, ia), muls(t10, a));
    v3 bot = add(muls(t01, ia), muls(t11, a));
    return add(muls(top, ib), muls(bot, b));
}

/* get_col, :259-345.  Returns rgb; *n_rk = completed RK updates; *fate = BH_FATE_*;
 * final_state (optional): ro, rd at exit. */
static v3 get_col_state(const params* P, const sky_t* S, v3 ro0, v3 rd0, uint32_t* n_rk, uint32_t* fate,
                        float* final_state) {
    v3 ro = ro0, rd = rd0;
    v3 c = cross(ro, rd);                       /* :262 */
    float h2 = dot(c, c);                       /* :263 */
    float distance_travelled = 0.0f;            /* :264 */
    int outside = 0;                            /* :265 */
    v3 nro0 = normalize(ro0);
    v3 cps = muls(muls(mk(-nro0.x, -nro0.y, -nro0.z), 1.5f), P->RS); /* :294, (-n * 1.5) * RS */
    uint32_t i;
    *fate = BH_FATE_CAP;
#define FINAL() do { if (final_state) { final_state[0] = ro.x; final_state[1] = ro.y; final_state[2] = ro.z; \
                     final_state[3] = rd.x; final_state[4] = rd.y; final_state[5] = rd.z; } } while (0)
    for (i = 0; i < P->max_iters; i++) {        /* :266 */
        float r = len(ro);                      /* :271 */
        if (P->BLACKOUT_EH != 0u) {             /* :272-283 */
            if (r < 1.0f) {
                if (dot(rd, ro) < 0.0f) { *n_rk = i; *fate = BH_FATE_BLACKOUT; FINAL(); return mk(0, 0, 0); }
            }
            if (r > 1.0f) outside = 1;
            else if (outside) { *n_rk = i; *fate = BH_FATE_BLACKOUT; FINAL(); return mk(0, 0, 0); }
        }
        float ds = sdf(P, ro);                  /* :285 */
        if (ds < MIN_DIST) { *n_rk = i; *fate = BH_FATE_SURFACE; FINAL(); return mk(1, 1, 1); } /* :286-288 */
        float dps = sdf_sphere(ro, cps, 0.075f);/* :294 */
        float dist = fminf(ds, dps);            /* :299 */
        float dd = P->DTM * r;                  /* :307 */
        dd = fminf(dist * 0.9f, dd);            /* :310 */
        v3 dro, drd;
        rk4(P, ro, rd, dd, h2, &dro, &drd);     /* :313 */
        ro = add(ro, dro);                      /* :315 */
        rd = add(rd, drd);                      /* :322 */
        distance_travelled += dd;               /* :324 */
        if (distance_travelled > P->MAX_DIST) { i++; *fate = BH_FATE_ESCAPE; break; } /* :325-327 */
    }
    *n_rk = i;
    FINAL();
#undef FINAL
    v3 n = normalize(rd);                                       /* :330 */
    float az = (P->variant & BHO_V_ATAN2F) ? atan2f(n.z, n.x)
                                           : (float)atan2((double)n.z, (double)n.x); /* :332 */
    float x = (az + ONE_PI) / TWO_PI;                           /* :334 */
    float y = (n.y + 1.0f) * 0.5f;                              /* :336 */
    v3 col = sample_bilinear(S, x, 1.0f - y);                   /* :341 */
    col.y = powv(col.y, 1.5f, P->variant);                      /* :342 */
    col.z = powv(col.z, 1.5f, P->variant);                      /* :343 */
    return col;
}
static v3 get_col(const params* P, const sky_t* S, v3 ro0, v3 rd0, uint32_t* n_rk, uint32_t* fate) {
    return get_col_state(P, S, ro0, rd0, n_rk, fate, 0);
}

/* sRGB -> linear decode of an 8-bit unorm (Rgba8UnormSrgb), computed in double. */
void bho_srgb_lut(float lut[256]) {
    for (int i = 0; i < 256; i++) {
        double c = (double)i / 255.0;
        lut[i] = (float)(c <= 0.04045 ? c / 12.92 : pow((c + 0.055) / 1.055, 2.4));
    }
}

/* Linear -> sRGB 8-bit store (Bgra8UnormSrgb), normative: clamp, OETF in double, round half up. */
uint8_t bho_srgb_encode(float x) {
    if (!(x > 0.0f)) return 0;          /* also NaN -> 0 */
    if (x >= 1.0f) return 255;
    double v = (double)x;
    double s = v <= 0.0031308 ? 12.92 * v : 1.055 * pow(v, 1.0 / 2.4) - 0.055;
    double q = floor(s * 255.0 + 0.5);
    return (uint8_t)(q > 255.0 ? 255.0 : q);
}

/* The encode over an array (test helper: the BGRA8 output's expected bytes). */
void bho_srgb_encode_array(const float* x, uint8_t* out, size_t n, int threads) {
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < (long long)n; i++) out[i] = bho_srgb_encode(x[i]);
}

/* Test helper: the number of floats x in [0, 1] (every bit pattern 0 .. 0x3F800000) whose
 * threshold-table code (largest k with x >= T[k], T[0] = 0, T[256] = +inf) differs from
 * bho_srgb_encode(x) -- i.e. checks a 257-entry threshold table against the definition. */
uint64_t bho_srgb_table_mismatches(const float T[257], int threads) {
    uint64_t bad = 0;
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static) reduction(+ : bad)
    for (long long b = 0; b <= 0x3F800000LL; b++) {
        float x;
        uint32_t u = (uint32_t)b;
        memcpy(&x, &u, 4);
        int lo = 0, hi = 256;  /* largest k in [0, 255] with x >= T[k] */
        while (hi - lo > 1) {
            int mid = (lo + hi) / 2;
            if (x >= T[mid]) lo = mid; else hi = mid;
        }
        bad += (uint8_t)lo != bho_srgb_encode(x);
    }
    return bad;
}

/* vs_main + rasteriser + fs_main ray setup (:37-55, :360-363): the per-vertex world ray vectors are
 * interpolated at the pixel centre with barycentrics of the fixed screen triangle
 * (3,1), (-1,1), (-1,-3) (src/uniforms.rs:114-118):  l0 = (x+.5)/(2W), l2 = (y+.5)/(2H), l1 = 1-l0-l2. */
static v3 pixel_dir(const bh_camera_uniform* cam, uint32_t W, uint32_t H, uint32_t px, uint32_t py) {
    float l0 = ((float)px + 0.5f) / (2.0f * (float)W);
    float l2 = ((float)py + 0.5f) / (2.0f * (float)H);
    float l1 = (1.0f - l0) - l2;
    v3 c0 = mk(cam->world_tri[0][0], cam->world_tri[0][1], cam->world_tri[0][2]);
    v3 c1 = mk(cam->world_tri[1][0], cam->world_tri[1][1], cam->world_tri[1][2]);
    v3 c2 = mk(cam->world_tri[2][0], cam->world_tri[2][1], cam->world_tri[2][2]);
    return add(add(smul(l0, c0), smul(l1, c1)), smul(l2, c2));
}

int bho_screen_tri_is_default(const bh_camera_uniform* cam) {
    static const float st[3][2] = {{3.0f, 1.0f}, {-1.0f, 1.0f}, {-1.0f, -3.0f}};
    for (int i = 0; i < 3; i++)
        if (cam->screen_tri[i][0] != st[i][0] || cam->screen_tri[i][1] != st[i][1]) return 0;
    return 1;
}

/*
 * Render rows row0, row0 + row_step, ... (< row1) of a width x height frame (row_step 0 == 1).
 * Outputs are row-major over the rendered rows, nrows = ceil((row1-row0)/row_step):
 * out_col / out_blackout: nrows*width*4 floats (RGBA, alpha = 1; blackout may be NULL);
 * n_rk (u16) / fate (u8): one per pixel, may be NULL.  threads <= 0: OpenMP default.
 * Returns 0, or -1 on invalid arguments.
 */
static int render_rows_v(uint32_t variant, const bh_camera_uniform* cam, const bh_uniforms* U, const uint8_t* sky,
                    uint32_t sky_w, uint32_t sky_h, uint32_t width, uint32_t height,
                    uint32_t max_iters, uint32_t scene_flags, uint32_t row0, uint32_t row1,
                    uint32_t row_step, float* out_col, float* out_blackout, uint16_t* n_rk, uint8_t* fate,
                    int threads) {
    if (!cam || !U || !sky || !out_col || sky_w == 0 || sky_h == 0 || width == 0 || height == 0 ||
        row0 > row1 || row1 > height || max_iters == 0 || max_iters > 65535u)
        return -1;
    if (!bho_screen_tri_is_default(cam)) return -2;
    params P;
    P.RS = U->rs; P.DTM = U->delta_time_mult; P.MAX_DIST = U->max_dist; P.DP = U->distortion_power;
    P.BLACKOUT_EH = U->blackout_eh; P.flags = scene_flags; P.max_iters = max_iters; P.variant = variant;
    sky_t S;
    S.tex = sky; S.w = sky_w; S.h = sky_h; S.variant = variant;
    bho_srgb_lut(S.lut);
    v3 ro0 = mk(cam->pos[0], cam->pos[1], cam->pos[2]);
    if (row_step == 0) row_step = 1;
    long nrows = ((long)row1 - (long)row0 + (long)row_step - 1) / (long)row_step;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#else
    (void)threads;
#endif
    for (long rr = 0; rr < nrows; rr++) {
        uint32_t py = row0 + (uint32_t)rr * row_step;
        for (uint32_t px = 0; px < width; px++) {
            size_t o = (size_t)rr * width + px;
            v3 rd0 = normalize(pixel_dir(cam, width, height, px, py)); /* :362 */
            uint32_t nrk, ft;
            v3 col = get_col(&P, &S, ro0, rd0, &nrk, &ft);           /* :364 */
            out_col[4 * o + 0] = col.x; out_col[4 * o + 1] = col.y;
            out_col[4 * o + 2] = col.z; out_col[4 * o + 3] = 1.0f;
            if (out_blackout) {                                      /* :365-368 */
                int keep = !(dot(col, col) < 1.0f);
                out_blackout[4 * o + 0] = keep ? col.x : 0.0f;
                out_blackout[4 * o + 1] = keep ? col.y : 0.0f;
                out_blackout[4 * o + 2] = keep ? col.z : 0.0f;
                out_blackout[4 * o + 3] = 1.0f;
            }
            if (n_rk) n_rk[o] = (uint16_t)nrk;
            if (fate) fate[o] = (uint8_t)ft;
        }
    }
    return 0;
}

int bho_render_rows(const bh_camera_uniform* cam, const bh_uniforms* U, const uint8_t* sky,
                    uint32_t sky_w, uint32_t sky_h, uint32_t width, uint32_t height,
                    uint32_t max_iters, uint32_t scene_flags, uint32_t row0, uint32_t row1,
                    uint32_t row_step, float* out_col, float* out_blackout, uint16_t* n_rk, uint8_t* fate,
                    int threads) {
    return render_rows_v(0u, cam, U, sky, sky_w, sky_h, width, height, max_iters, scene_flags, row0, row1, row_step, out_col, out_blackout, n_rk, fate, threads);
}

/* bho_render_rows with a parity-envelope variant (BHO_V_* bits; test infrastructure for DESIGN.md §3). */
int bho_render_rows_variant(const bh_camera_uniform* cam, const bh_uniforms* U, const uint8_t* sky,
                    uint32_t sky_w, uint32_t sky_h, uint32_t width, uint32_t height,
                    uint32_t max_iters, uint32_t scene_flags, uint32_t row0, uint32_t row1,
                    uint32_t row_step, float* out_col, float* out_blackout, uint16_t* n_rk, uint8_t* fate,
                    int threads, uint32_t variant) {
    return render_rows_v(variant, cam, U, sky, sky_w, sky_h, width, height, max_iters, scene_flags, row0, row1, row_step, out_col, out_blackout, n_rk, fate, threads);
}

/* Trace one pixel (debug/KAT helper): writes final ro, rd (6 floats) too. */
int bho_trace_pixel(const bh_camera_uniform* cam, const bh_uniforms* U, const uint8_t* sky,
                    uint32_t sky_w, uint32_t sky_h, uint32_t width, uint32_t height,
                    uint32_t max_iters, uint32_t scene_flags, uint32_t px, uint32_t py,
                    float out_rgb[3], uint32_t* n_rk, uint32_t* fate) {
    if (px >= width || py >= height) return -1;
    params P;
    P.RS = U->rs; P.DTM = U->delta_time_mult; P.MAX_DIST = U->max_dist; P.DP = U->distortion_power;
    P.BLACKOUT_EH = U->blackout_eh; P.flags = scene_flags; P.max_iters = max_iters; P.variant = 0;
    sky_t S;
    S.tex = sky; S.w = sky_w; S.h = sky_h; S.variant = 0;
    bho_srgb_lut(S.lut);
    v3 ro0 = mk(cam->pos[0], cam->pos[1], cam->pos[2]);
    v3 rd0 = normalize(pixel_dir(cam, width, height, px, py));
    v3 col = get_col(&P, &S, ro0, rd0, n_rk, fate);
    out_rgb[0] = col.x; out_rgb[1] = col.y; out_rgb[2] = col.z;
    return 0;
}

/* Integrate one explicit ray (ro0, rd0 not necessarily from a camera) — physics KATs.
 * out_state (optional, 6 floats): final ro, rd. */
int bho_trace_ray(const float ro0_in[3], const float rd0_in[3], const bh_uniforms* U,
                  const uint8_t* sky, uint32_t sky_w, uint32_t sky_h, uint32_t max_iters,
                  uint32_t scene_flags, float out_rgb[3], uint32_t* n_rk, uint32_t* fate, float* out_state) {
    params P;
    P.RS = U->rs; P.DTM = U->delta_time_mult; P.MAX_DIST = U->max_dist; P.DP = U->distortion_power;
    P.BLACKOUT_EH = U->blackout_eh; P.flags = scene_flags; P.max_iters = max_iters; P.variant = 0;
    sky_t S;
    S.tex = sky; S.w = sky_w; S.h = sky_h; S.variant = 0;
    bho_srgb_lut(S.lut);
    v3 col = get_col_state(&P, &S, mk(ro0_in[0], ro0_in[1], ro0_in[2]), mk(rd0_in[0], rd0_in[1], rd0_in[2]),
                           n_rk, fate, out_state);
    out_rgb[0] = col.x; out_rgb[1] = col.y; out_rgb[2] = col.z;
    return 0;
}
