// bh_host.cpp — C ABI of include/bh_render.h: context, camera/uniform host math, synthetic sky,
// render dispatch.  No CPU rendering path exists here by design: bh_render runs the HIP kernel or
// fails with a status code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "bh_common.hpp"
#include "bh_srgb.hpp"

struct bh_ctx {
    int device = 0;
    uint32_t* sky = nullptr;       // device RGBA8 texels
    float* lut = nullptr;          // device sRGB->linear table (256 floats)
    float* enc = nullptr;          // device linear->sRGB threshold table (257 floats)
    uint8_t* enc_b = nullptr;      // device base codes of the table-form encoder (SRGB_BUCKETS bytes)
    uint32_t* enc_e = nullptr;     // device code table of the code-table encoder (SRGB_CODES words)
    uint32_t* counters = nullptr;  // persistent-schedule work counters (1 KiB, zeroed per launch)
    uint32_t sky_w = 0, sky_h = 0;
    uint32_t grid_exact = 0, grid_fast = 0;  // resident blocks of the persistent kernels
    uint32_t cus = 0;                        // compute units of the device
    // temporal dispatch order (tile schedule): per-tile cost of the previous frame -> order, one state
    // per (frame geometry, shard, stream).  Never freed before bh_destroy except by LRU eviction beyond
    // BH_ORDER_STATES states, so a graph captured after the first call of a key keeps valid pointers,
    // and renders on different streams (frames in flight) never share costs or counters.
    struct OrderState {
        uint32_t width = 0, height = 0, shard_index = 0, shard_count = 0;
        uint64_t partition = 0;              // bh_partition::serial, 0 = none
        uint64_t n_tiles = 0;                // the buffers' size in tiles
        void* stream = nullptr;
        uint64_t last_use = 0;
        bool valid = false;                  // costs and histogram agree (false: start afresh)
        bool captured = false;               // used by a launch captured into a graph: never evicted
        // Which frames the buffers describe (frame_cost_key): the costs in tile_cost (and the histogram the
        // counters hold of them, always pending) are those of a frame with key cost_key; the current order
        // was built from costs with key order_key.  A launch whose frame 0 has the key of both (a repeated
        // frame: a fixed camera) needs neither the order build nor new costs -- the march's step counts, and
        // so the costs, are a function of that key.
        uint64_t cost_key = 0, order_key = ~0ull;
        uint8_t* tile_cost = nullptr;
        uint32_t* order = nullptr;
        uint32_t* counters = nullptr;        // ORDER_WORDS words (bh_common.hpp)
    };
    std::vector<OrderState> orders;
    uint64_t order_clock = 0;
    // per-frame arguments of bh_render_frames calls of more than BH_INLINE_FRAMES frames, one table per
    // stream: the kernels of one stream run in order, so one device table serves every call on it; the
    // host writes a pinned slot of a ring and copies it in on the stream (the slot is reused once its
    // copy has run: its event)
    static constexpr uint32_t FRAME_RING = 4;
    struct FrameTable {
        void* stream = nullptr;
        bh::FrameArgs* dev = nullptr;                 // BH_MAX_FRAMES entries
        bh::FrameArgs* host[FRAME_RING] = {};         // pinned, BH_MAX_FRAMES entries each
        hipEvent_t done[FRAME_RING] = {};             // the slot's copy has executed
        uint32_t next = 0;
        std::vector<bh::FrameArgs> last;              // what the table holds once the stream's copies ran
    };
    std::vector<FrameTable> frame_tables;
    // post-processing (bh_bloom) scratch: one set of textures per (width, height, levels), with the
    // separable plans of its up passes (sep_plan).  Graph contract as the order states: a set used under
    // stream capture is never evicted (bh_graph_release clears the mark); others are evicted least
    // recently used beyond BH_BLOOM_SETS.
    // ext: the largest block footprint side (up passes); nc, nr: the inexact columns / rows (same plan)
    // host: the plan's host copy in bh_bloom_check's dry mode (dev then points into it; never freed as device memory)
    struct SepPlan {
        std::array<uint32_t, 8> key{};  // ow, oh, tw, th, rx, ry, grid origin, in-block fix
        uint32_t* dev = nullptr;
        int ext = 0;
        uint32_t nc = 0, nr = 0;
        // same-size plan: the quad grid origin of the in-block fix and its residual (crossing) columns / rows,
        // listed after the full list
        uint32_t org = 0, nrc = 0, nrr = 0, nrc2 = 0, nrr2 = 0;  // residual lists of the Y / final epilogue
        size_t rec = 0;  // word offset of the lists' fix-up records (full, residual 1, residual 2; 8 words each)
        // the final epilogue's column strips (bh_bloom_strip_table): word offset of the table (0: none), its
        // strip columns and the strip storage (3 images x stw columns x oh rows; not allocated in dry mode)
        size_t stc = 0;
        uint32_t stw = 0;
        uint32_t* strips = nullptr;
        std::shared_ptr<std::vector<uint32_t>> host;
    };
    struct BloomScratch {
        uint64_t key = 0;
        std::vector<uint32_t*> tex;
        std::vector<SepPlan> sep_plans;
        uint32_t prepared = 0;   // bit s: schedule s ran once outside capture (every plan it uses exists)
        bool captured = false;
        uint64_t last_use = 0;
    };
    std::vector<BloomScratch> blooms;
    uint64_t bloom_clock = 0;
    // shader-clock probe of the march launches (bh_set_clock_probe): device accumulators or null
    unsigned long long* clk = nullptr;
    uint32_t clk_mask = 0;
};

// A weighted tile partition (include/bh_render.h, bh_partition_create).
struct bh_partition {
    uint32_t width = 0, height = 0, shard_count = 0, tiles_x = 0, tiles_y = 0;
    int device = 0;
    std::vector<uint32_t> count, offset;  // per shard: tiles, first entry in tile_list
    uint32_t* tile_list = nullptr;        // device: every shard's tiles in packed order (tx | ty << 16)
    uint32_t* tile_loc = nullptr;         // device: per tile (ty * tiles_x + tx): packed index | shard << 24
    uint64_t serial = 0;                  // unique per created partition: the temporal-order key (an
                                          // address can be reused by a later partition)
};
static std::atomic<uint64_t> g_partition_serial{0};
static void free_frame_table(bh_ctx::FrameTable& t);
static void free_bloom_scratch(bh_ctx::BloomScratch& b) {
    for (uint32_t* t : b.tex) (void)hipFree(t);
    for (auto& p : b.sep_plans)
        if (!p.host) {
            (void)hipFree(p.dev);
            (void)hipFree(p.strips);
        }
    b.tex.clear();
    b.sep_plans.clear();
}
// True when `s` is capturing -- or when the runtime cannot say (e.g. the legacy stream while another
// stream captures in global mode): the callers then refuse to allocate, which a capture would not survive.
static bool stream_capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
}

namespace {

thread_local std::string g_last_error;
// a validation failure without its own message: name the entry point and the check's line
static int bad_arg(const char* fn, int line) {
    g_last_error = std::string(fn) + ": invalid argument (bh_host.cpp:" + std::to_string(line) + ")";
    return BH_ERR_INVALID_ARG;
}

int hip_fail(hipError_t e, const char* what) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return BH_ERR_HIP;
}

// Makes `device` current for one ABI call and restores the caller's device on every return path.
struct DeviceScope {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceScope(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != device) err = hipSetDevice(device);
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};

// ---- glam 0.24 Vec3 subset (scalar f32, left-to-right association as glam writes it) ----------
struct V3 { float x, y, z; };
V3 v_add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V3 v_sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 v_mul(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
float v_dot(V3 a, V3 b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); }
V3 v_cross(V3 a, V3 b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
V3 v_normalize(V3 a) { return v_mul(a, 1.0f / std::sqrt(v_dot(a, a))); }  // self * length_recip()
V3 v_neg(V3 a) { return {-a.x, -a.y, -a.z}; }

// sRGB byte -> linear, in double (the Rgba8UnormSrgb decode; DESIGN.md "Normative arithmetic").
void srgb_lut(float lut[256]) {
    for (int i = 0; i < 256; ++i) {
        double c = (double)i / 255.0;
        lut[i] = (float)(c <= 0.04045 ? c / 12.92 : std::pow((c + 0.055) / 1.055, 2.4));
    }
}

// linear -> sRGB byte of a Bgra8UnormSrgb store: clamp to [0, 1] (NaN -> 0), the sRGB OETF in double,
// round half up (the normative encode, DESIGN.md "Output formats").
uint8_t srgb_encode_ref(float x) {
    if (!(x > 0.0f)) return 0;
    if (x >= 1.0f) return 255;
    const double v = (double)x;
    const double e = v <= 0.0031308 ? 12.92 * v : 1.055 * std::pow(v, 1.0 / 2.4) - 0.055;
    const double q = std::floor(e * 255.0 + 0.5);
    return (uint8_t)(q > 255.0 ? 255.0 : q);
}

// Thresholds of the encode (bh_srgb.hpp): T[k] = the smallest float in (0, 1] with code >= k,
// found by bisection over the ordered bit patterns of positive floats.
void srgb_encode_table(float T[257]) {
    T[0] = 0.0f;
    for (int k = 1; k < 256; ++k) {
        uint32_t lo = 0u, hi = 0x3F800000u;  // code(lo) < k <= code(hi)
        while (hi - lo > 1u) {
            const uint32_t mid = lo + (hi - lo) / 2u;
            float x;
            std::memcpy(&x, &mid, 4);
            if (srgb_encode_ref(x) >= k) hi = mid; else lo = mid;
        }
        std::memcpy(&T[k], &hi, 4);
    }
    T[256] = std::numeric_limits<float>::infinity();
}

}  // namespace

// The code-table form of the encoder (bh_srgb.hpp srgb_encode_code): false if a bucket held two thresholds
// (never, for the normative table: the form would not be exact).
extern "C" __attribute__((visibility("hidden"))) bool bh_srgb_code_table(const float* T, uint32_t* E) {
    bool ok = true;
    for (int i = 0; i < bh::SRGB_CODES; ++i) {
        const uint32_t hi = (bh::SRGB_BUCKET_BASE + (uint32_t)i) << bh::SRGB_BUCKET_SHIFT;
        float lo;
        std::memcpy(&lo, &hi, 4);
        int k = 0;  // code of the bucket's lower end
        while (k < 255 && lo >= T[k + 1]) ++k;
        uint32_t thr = 0x10000u;
        if (k < 255) {
            uint32_t tb;
            std::memcpy(&tb, &T[k + 1], 4);
            if ((tb >> 16) == (hi >> 16)) {
                thr = tb & 0xFFFFu;
                uint32_t t2 = 0;
                if (k < 254) std::memcpy(&t2, &T[k + 2], 4);
                if (k < 254 && (t2 >> 16) == (hi >> 16)) ok = false;
            }
        }
        if (i == 0 && thr != 0x10000u) ok = false;  // values below 2^-13 clamp to entry 0
        E[i] = (uint32_t)k | (thr << 15);
    }
    return ok;
}

extern "C" __attribute__((visibility("hidden"))) void bh_srgb_bucket_table(const float* T, uint8_t* B) {
    for (int i = 0; i < bh::SRGB_BUCKETS; ++i) {
        const uint32_t bits = (bh::SRGB_BUCKET_BASE + (uint32_t)i) << bh::SRGB_BUCKET_SHIFT;
        float lo;
        std::memcpy(&lo, &bits, 4);
        int k = 0;  // code of the bucket's lower end: the largest k with T[k] <= lo
        while (k < 255 && lo >= T[k + 1]) ++k;
        B[i] = (uint8_t)k;
    }
}

namespace {

// Screen row (in tiles) of the black hole's projection: solve C1 + l0 (C0 - C1) + l2 (C2 - C1) = -t ro0
// (t > 0) for the barycentrics of the pixel looking at the origin; py = 2 H l2 - 0.5.  Falls back to
// the middle row when the origin is behind the camera or the system is degenerate.
uint32_t bh_tile_row(const bh_camera_uniform* c, uint32_t height) {
    const double C0[3] = {c->world_tri[0][0], c->world_tri[0][1], c->world_tri[0][2]};
    const double C1[3] = {c->world_tri[1][0], c->world_tri[1][1], c->world_tri[1][2]};
    const double C2[3] = {c->world_tri[2][0], c->world_tri[2][1], c->world_tri[2][2]};
    const double A[3] = {C0[0] - C1[0], C0[1] - C1[1], C0[2] - C1[2]};
    const double B[3] = {C2[0] - C1[0], C2[1] - C1[1], C2[2] - C1[2]};
    const double P[3] = {c->pos[0], c->pos[1], c->pos[2]};  // l0 A + l2 B + t P = -C1
    auto det3 = [](const double* x, const double* y, const double* z) {
        return x[0] * (y[1] * z[2] - y[2] * z[1]) - y[0] * (x[1] * z[2] - x[2] * z[1]) + z[0] * (x[1] * y[2] - x[2] * y[1]);
    };
    const double R[3] = {-C1[0], -C1[1], -C1[2]};
    const double D = det3(A, B, P);
    const uint32_t tiles_y = (height + 7u) / 8u;
    if (std::fabs(D) < 1e-12) return tiles_y / 2u;
    const double l2 = det3(A, R, P) / D, t = det3(A, B, R) / D;
    if (!(t > 0.0)) return tiles_y / 2u;
    double py = 2.0 * height * l2 - 0.5;
    py = py < 0.0 ? 0.0 : (py > height - 1.0 ? height - 1.0 : py);
    return (uint32_t)(py / 8.0);
}

bool screen_tri_default(const bh_camera_uniform* c) {
    static const float st[3][2] = {{3.0f, 1.0f}, {-1.0f, 1.0f}, {-1.0f, -3.0f}};
    for (int i = 0; i < 3; ++i)
        if (c->screen_tri[i][0] != st[i][0] || c->screen_tri[i][1] != st[i][1]) return false;
    return true;
}

uint64_t splitmix64(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint64_t hash3(uint64_t seed, int64_t a, int64_t b, int64_t c) {
    uint64_t s = seed ^ ((uint64_t)a * 0x9E3779B185EBCA87ull) ^ ((uint64_t)b * 0xC2B2AE3D27D4EB4Full) ^
                 ((uint64_t)c * 0x165667B19E3779F9ull);
    return splitmix64(s);
}
float unit(uint64_t h) { return (float)(h >> 40) * (1.0f / 16777216.0f); }

// periodic-in-x lattice value noise, smoothstep interpolation
float value_noise(uint64_t seed, int oct, float x, float y, int period_x) {
    float fx = std::floor(x), fy = std::floor(y);
    int ix = (int)fx, iy = (int)fy;
    float tx = x - fx, ty = y - fy;
    tx = tx * tx * (3.0f - 2.0f * tx);
    ty = ty * ty * (3.0f - 2.0f * ty);
    auto L = [&](int cx, int cy) {
        int wx = ((cx % period_x) + period_x) % period_x;
        return unit(hash3(seed, oct, wx, cy));
    };
    float a = L(ix, iy), b = L(ix + 1, iy), c = L(ix, iy + 1), d = L(ix + 1, iy + 1);
    return (a + (b - a) * tx) + ((c + (d - c) * tx) - (a + (b - a) * tx)) * ty;
}

uint8_t encode8(float lin) {
    if (!(lin > 0.0f)) return 0;
    if (lin >= 1.0f) return 255;
    double v = lin, s = v <= 0.0031308 ? 12.92 * v : 1.055 * std::pow(v, 1.0 / 2.4) - 0.055;
    return (uint8_t)std::floor(s * 255.0 + 0.5);
}

}  // namespace

extern "C" {

int bh_abi_version(void) { return BH_ABI_VERSION; }

// for the other host translation units (bh_present.cpp)
__attribute__((visibility("hidden"))) void bh_set_last_error(const std::string& msg) { g_last_error = msg; }
__attribute__((visibility("hidden"))) int bh_bad_arg(const char* fn, int line) {
    g_last_error = std::string(fn) + ": invalid argument (line " + std::to_string(line) + ")";
    return BH_ERR_INVALID_ARG;
}
__attribute__((visibility("hidden"))) int bh_ctx_device(const bh_ctx* c) { return c->device; }

const char* bh_status_string(int st) {
    switch (st) {
        case BH_OK: return "ok";
        case BH_ERR_INVALID_ARG: return "invalid argument";
        case BH_ERR_UNSUPPORTED: return "unsupported";
        case BH_ERR_HIP: return "HIP runtime error";
        case BH_ERR_NO_DEVICE: return "no HIP device";
        case BH_ERR_OUT_OF_MEMORY: return "out of device memory";
        case BH_ERR_INTERNAL: return "internal consistency check failed";
        default: return "unknown status";
    }
}

const char* bh_last_error(void) { return g_last_error.c_str(); }

// Scene::new defaults, src/scene.rs:89-137 (RS 1.0, max dt 0.5, bg 0.5, blackout PodBool::r#false()
// whose inner is 1 (src/podbool.rs:24-26), max dist 250, distortion 1.0); 24 B padded to 32.
int bh_srgb_encode_table(float* out257) {
    if (!out257) return bad_arg(__func__, __LINE__);
    srgb_encode_table(out257);
    return BH_OK;
}

int bh_uniforms_default(bh_uniforms* out) {
    if (!out) return bad_arg(__func__, __LINE__);
    std::memset(out, 0, sizeof(*out));
    out->rs = 1.0f;
    out->delta_time_mult = 0.5f;
    out->bg_brightness = 0.5f;
    out->blackout_eh = 1u;
    out->max_dist = 250.0f;
    out->distortion_power = 1.0f;
    return BH_OK;
}

// src/scene.rs:68-76
int bh_camera_default(uint32_t width, uint32_t height, bh_camera* out) {
    if (!out || width == 0 || height == 0) return bad_arg(__func__, __LINE__);
    const float PI = 3.14159265358979323846f;  // std::f32::consts::PI
    *out = bh_camera{{0.0f, 0.0f, -20.0f}, {0.0f, 0.0f, 1.0f}, {0.0f, 1.0f, 0.0f},
                     (float)width / (float)height, PI * 0.5f, 0.1f, 100.0f};
    return BH_OK;
}

}  // extern "C"

namespace {
// glam 0.24 Quat (f32): from_axis_angle and mul_vec3 (the SSE2 path evaluates the same formula with
// the same operand order: dot = (x + y) + z, no FMA)
struct Q4 { float x, y, z, w; };
Q4 q_from_axis_angle(V3 axis, float angle) {
    const float h = angle * 0.5f;
    const float s = std::sin(h), c = std::cos(h);  // f32::sin_cos
    const V3 v = v_mul(axis, s);
    return {v.x, v.y, v.z, c};
}
V3 q_mul_vec3(Q4 q, V3 rhs) {
    const float w = q.w;
    const V3 b{q.x, q.y, q.z};
    const float b2 = v_dot(b, b);
    return v_add(v_add(v_mul(rhs, w * w - b2), v_mul(b, v_dot(rhs, b) * 2.0f)), v_mul(v_cross(b, rhs), w * 2.0f));
}
float axis_norm(uint8_t neg, uint8_t pos) { return (neg == pos) ? 0.0f : (pos ? 1.0f : -1.0f); }
}  // namespace

extern "C" {

int bh_controller_update(const bh_controller* k, bh_camera* cam, float dt, int do_pan, int* moved) {
    if (!k || !cam) return bad_arg(__func__, __LINE__);
    V3 pos{cam->pos[0], cam->pos[1], cam->pos[2]};
    V3 dir{cam->dir[0], cam->dir[1], cam->dir[2]};
    V3 up{cam->up[0], cam->up[1], cam->up[2]};
    auto right = [&] { return v_cross(up, dir); };  // Camera::right = up x dir (camera.rs:32)
    const float xn = axis_norm(k->left, k->right), zn = axis_norm(k->backward, k->forward);
    const float yn = axis_norm(k->down, k->up);
    const float xm = dt * k->speed * xn, zm = dt * k->speed * zn, ym = dt * k->speed * yn;
    pos = v_add(pos, v_mul(right(), xm));
    pos = v_add(pos, v_mul(dir, zm));
    pos = v_add(pos, v_mul(up, ym));
    const float en = axis_norm(k->exp_towards_origin, k->exp_away_origin);
    pos = v_mul(pos, std::exp(-dt * en));
    const float xpn = axis_norm(k->pan_left, k->pan_right), ypn = axis_norm(k->pan_up, k->pan_down);
    const float xp = dt * k->pan_speed * xpn, yp = dt * k->pan_speed * ypn;
    auto rotate = [&](V3 axis, float angle) {
        const Q4 q = q_from_axis_angle(axis, angle);
        dir = q_mul_vec3(q, dir);
        up = q_mul_vec3(q, up);
    };
    rotate(V3{0.0f, 1.0f, 0.0f}, xp);
    rotate(right(), yp);
    float mx = 0.0f, my = 0.0f;  // cursor_movement (camera.rs:268-278)
    if (k->has_prev_cursor && k->has_curr_cursor) {
        mx = k->curr_cursor[0] - k->prev_cursor[0];
        my = k->curr_cursor[1] - k->prev_cursor[1];
    }
    const float ps = dt * k->pan_speed;
    if (k->mouse_pressed && do_pan) {
        rotate(V3{0.0f, 1.0f, 0.0f}, ps * mx);
        rotate(right(), ps * my);
    }
    cam->pos[0] = pos.x; cam->pos[1] = pos.y; cam->pos[2] = pos.z;
    cam->dir[0] = dir.x; cam->dir[1] = dir.y; cam->dir[2] = dir.z;
    cam->up[0] = up.x; cam->up[1] = up.y; cam->up[2] = up.z;
    if (moved) *moved = (xn != 0.0f) | (yn != 0.0f) | (zn != 0.0f) | (xpn != 0.0f) | (ypn != 0.0f);
    return BH_OK;
}

int bh_camera_look_at(const float pos[3], const float target[3], uint32_t width, uint32_t height,
                      bh_camera* out) {
    if (!pos || !target) return bad_arg(__func__, __LINE__);
    int st = bh_camera_default(width, height, out);
    if (st != BH_OK) return st;
    V3 p{pos[0], pos[1], pos[2]}, t{target[0], target[1], target[2]};
    V3 d = v_normalize(v_sub(t, p));
    std::memcpy(out->pos, pos, 3 * sizeof(float));
    out->dir[0] = d.x; out->dir[1] = d.y; out->dir[2] = d.z;
    return BH_OK;
}

// CameraUniform::new (src/uniforms.rs:108-122) + ::update (:123-133) ->
// Camera::pos_to_world_space_screen_triangle (src/camera.rs:89-112):
//   corner_i = rot_matrix * ( -(tx * cx_i), -(-ty) * cy_i ... ) — concretely
//   dir_camera = -vec3(tx*cx, -ty*cy, 1)  (camera.rs:70-74),
//   rot_matrix = look_at_rh(pos, pos + dir, up).inverse()  (camera.rs:56-58),
//   world = rot_matrix.transform_vector3(dir_camera)  (camera.rs:76).
// The view matrix is a rigid transform, so its inverse's rotation block is the transpose
// (columns s, u, -f).  glam's general f32 Mat4::inverse may differ from the transpose in the last
// ulp; the corners are kernel INPUTS, so this host step is outside kernel parity.
int bh_camera_uniform_update(const bh_camera* cam, bh_camera_uniform* out) {
    if (!cam || !out) return bad_arg(__func__, __LINE__);
    std::memset(out, 0, sizeof(*out));
    static const float st[3][2] = {{3.0f, 1.0f}, {-1.0f, 1.0f}, {-1.0f, -3.0f}};
    for (int i = 0; i < 3; ++i) { out->screen_tri[i][0] = st[i][0]; out->screen_tri[i][1] = st[i][1]; }
    V3 pos{cam->pos[0], cam->pos[1], cam->pos[2]};
    V3 dir{cam->dir[0], cam->dir[1], cam->dir[2]};
    V3 up{cam->up[0], cam->up[1], cam->up[2]};
    // look_at_rh(eye, center, up) = look_to_rh(eye, center - eye, up)
    V3 f = v_normalize(v_sub(v_add(pos, dir), pos));
    V3 s = v_normalize(v_cross(f, up));
    V3 u = v_cross(s, f);
    V3 col0 = s, col1 = u, col2 = v_neg(f);
    // tan_fov_half (camera.rs:60-63)
    float tfy = std::tan(cam->fovy / 2.0f);
    float tfx = tfy * cam->aspect;
    for (int i = 0; i < 3; ++i) {
        float cx = st[i][0], cy = st[i][1];
        V3 dc = v_neg(V3{tfx * cx, -tfy * cy, 1.0f});
        // transform_vector3: res = x_axis*x; res = y_axis*y + res; res = z_axis*z + res
        V3 res = v_mul(col0, dc.x);
        res = v_add(v_mul(col1, dc.y), res);
        res = v_add(v_mul(col2, dc.z), res);
        out->world_tri[i][0] = res.x; out->world_tri[i][1] = res.y; out->world_tri[i][2] = res.z;
        out->world_tri[i][3] = 0.0f;
    }
    out->pos[0] = pos.x; out->pos[1] = pos.y; out->pos[2] = pos.z;
    return BH_OK;
}

static void sky_rows(uint8_t* out, uint32_t w, uint32_t h, uint64_t seed, uint32_t y0, uint32_t y1) {
    const int base = 6;  // nebula lattice cells around the equator at octave 0
    for (uint32_t y = y0; y < y1; ++y) {
        for (uint32_t x = 0; x < w; ++x) {
            float u = ((float)x + 0.5f) / (float)w, v = ((float)y + 0.5f) / (float)h;
            float n1 = 0.0f, n2 = 0.0f, amp = 0.5f;
            for (int o = 0; o < 5; ++o) {
                int per = base << o;
                n1 += amp * value_noise(seed, o, u * per, v * (per / 2), per);
                n2 += amp * value_noise(seed ^ 0xA5A5A5A5ull, o, u * per, v * (per / 2), per);
                amp *= 0.5f;
            }
            float neb = std::fmax(0.0f, n1 - 0.45f) * 1.6f;
            float r = 0.012f + 0.55f * neb * neb + 0.10f * n2 * neb;
            float g = 0.010f + 0.22f * neb * n2;
            float b = 0.030f + 0.65f * neb * (1.0f - 0.5f * n2);
            uint64_t hs = hash3(seed ^ 0x5354415253ull, 99, x, y);  // "STARS"
            if ((hs & 0xFFFu) < 6u) {                                // ~0.15 % of texels
                float mag = unit(hs);
                float temp = unit(hs * 0x2545F4914F6CDD1Dull);
                float L = 0.25f + 0.75f * mag * mag;
                r += L * (0.8f + 0.2f * temp);
                g += L * 0.85f;
                b += L * (1.0f - 0.3f * temp);
            }
            uint8_t* p = out + ((size_t)y * w + x) * 4u;
            p[0] = encode8(r); p[1] = encode8(g); p[2] = encode8(b); p[3] = 255;
        }
    }
}

// Rows are independent, so the result does not depend on the thread count.
int bh_synthetic_sky(uint8_t* out, uint32_t w, uint32_t h, uint64_t seed) {
    if (!out || w == 0 || h == 0) return bad_arg(__func__, __LINE__);
    unsigned nt = std::thread::hardware_concurrency();
    nt = nt == 0 ? 1 : (nt > 16 ? 16 : nt);
    if (nt > h) nt = h;
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nt; ++t) {
        uint32_t y0 = (uint32_t)((uint64_t)h * t / nt), y1 = (uint32_t)((uint64_t)h * (t + 1) / nt);
        pool.emplace_back(sky_rows, out, w, h, seed, y0, y1);
    }
    for (auto& th : pool) th.join();
    return BH_OK;
}

int bh_create(const uint8_t* sky, uint32_t sky_w, uint32_t sky_h, int device, bh_ctx** out) {
    if (!sky || !out || sky_w == 0 || sky_h == 0 || sky_w > 32768u || sky_h > 32768u) return bad_arg(__func__, __LINE__);
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) { g_last_error = "no HIP device"; return BH_ERR_NO_DEVICE; }
    if (device < 0 || device >= ndev) { g_last_error = "device index out of range"; return BH_ERR_NO_DEVICE; }
    DeviceScope dev(device);
    if (dev.err != hipSuccess) return hip_fail(dev.err, "hipSetDevice");
    bh_ctx* c = new (std::nothrow) bh_ctx();
    if (!c) return BH_ERR_OUT_OF_MEMORY;
    c->device = device;
    c->sky_w = sky_w;
    c->sky_h = sky_h;
    const size_t bytes = (size_t)sky_w * sky_h * 4u;
    float lut[256], enc[257];
    uint8_t enc_b[bh::SRGB_BUCKETS];
    uint32_t enc_e[bh::SRGB_CODES];
    srgb_lut(lut);
    srgb_encode_table(enc);
    bh_srgb_bucket_table(enc, enc_b);
    if (!bh_srgb_code_table(enc, enc_e)) {
        g_last_error = "sRGB code table";
        delete c;
        return BH_ERR_UNSUPPORTED;
    }
    int st = BH_OK;
    if ((e = hipMalloc(&c->sky, bytes)) != hipSuccess) st = (e == hipErrorOutOfMemory) ? BH_ERR_OUT_OF_MEMORY : hip_fail(e, "hipMalloc(sky)");
    else if ((e = hipMalloc(&c->lut, sizeof(lut))) != hipSuccess) st = hip_fail(e, "hipMalloc(lut)");
    else if ((e = hipMemcpy(c->sky, sky, bytes, hipMemcpyHostToDevice)) != hipSuccess) st = hip_fail(e, "hipMemcpy(sky)");
    else if ((e = hipMemcpy(c->lut, lut, sizeof(lut), hipMemcpyHostToDevice)) != hipSuccess) st = hip_fail(e, "hipMemcpy(lut)");
    else if ((e = hipMalloc(&c->enc, sizeof(enc))) != hipSuccess) st = hip_fail(e, "hipMalloc(enc)");
    else if ((e = hipMemcpy(c->enc, enc, sizeof(enc), hipMemcpyHostToDevice)) != hipSuccess) st = hip_fail(e, "hipMemcpy(enc)");
    else if ((e = hipMalloc(&c->enc_b, sizeof(enc_b))) != hipSuccess) st = hip_fail(e, "hipMalloc(enc_b)");
    else if ((e = hipMemcpy(c->enc_b, enc_b, sizeof(enc_b), hipMemcpyHostToDevice)) != hipSuccess) st = hip_fail(e, "hipMemcpy(enc_b)");
    else if ((e = hipMalloc(&c->enc_e, sizeof(enc_e))) != hipSuccess) st = hip_fail(e, "hipMalloc(enc_e)");
    else if ((e = hipMemcpy(c->enc_e, enc_e, sizeof(enc_e), hipMemcpyHostToDevice)) != hipSuccess) st = hip_fail(e, "hipMemcpy(enc_e)");
    else if ((e = hipMalloc(&c->counters, 1024)) != hipSuccess) st = hip_fail(e, "hipMalloc(counters)");
    if (st == BH_OK) {
        int cus = 0;
        if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess || cus <= 0) {
            st = hip_fail(e, "hipDeviceGetAttribute(CU count)");
        } else {
            c->cus = (uint32_t)cus;
            c->grid_exact = (uint32_t)(cus * bh_march_blocks_per_cu_exact());
            c->grid_fast = (uint32_t)(cus * bh_march_blocks_per_cu_fast());
        }
    }
    if (st != BH_OK) { bh_destroy(c); return st; }
    *out = c;
    return BH_OK;
}

int bh_destroy(bh_ctx* c) {
    if (!c) return BH_OK;
    DeviceScope dev(c->device);
    if (c->sky) (void)hipFree(c->sky);
    if (c->lut) (void)hipFree(c->lut);
    if (c->enc) (void)hipFree(c->enc);
    if (c->enc_b) (void)hipFree(c->enc_b);
    if (c->enc_e) (void)hipFree(c->enc_e);
    if (c->counters) (void)hipFree(c->counters);
    for (auto& o : c->orders) {
        if (o.tile_cost) (void)hipFree(o.tile_cost);
        if (o.order) (void)hipFree(o.order);
        if (o.counters) (void)hipFree(o.counters);
    }
    for (auto& b : c->blooms) free_bloom_scratch(b);
    for (auto& t : c->frame_tables) free_frame_table(t);
    delete c;
    return BH_OK;
}

}  // extern "C"

namespace {

// A same-size pass (copy, the blur's same-size downsample, a remix input: n texels sampled at n pixels)
// is the identity on stored texels when every pixel's bilinear sample encodes back to its own texel's
// byte.  Along one axis pixel x samples texels x0, x1 = clamp(floor(t)), clamp(floor(t) + 1) with
// weights 1 - fa, fa (t = RN(RN((x + 0.5) / n) * n) - 0.5, sample()'s arithmetic); where t == x the
// weights are exactly 1 and 0, elsewhere (e.g. 51 of 1920 columns, 42 of 1080 rows) t misses x by a few
// ulps and the weight on the other texel is tiny but not 0.  Every rounding of the 2-D lerp is monotone
// in each texel (weights >= 0), so with texel (x, y) = D the result lies between the lerp with every
// other texel 0 and with every other texel 1 (the largest decoded value); when both bounds encode to D's
// own byte for every byte value, every weight class of the two axes and both channel kinds (sRGB colour,
// linear alpha k/255), the pass returns its input's bytes whatever the other texels are.  Powers of two
// (t == x everywhere) pass trivially.
struct AxisClass {
    float ia, fa;  // the weights on texels x0 and x1
    bool d0, d1;   // x0 == x, x1 == x
    bool operator==(const AxisClass& o) const { return ia == o.ia && fa == o.fa && d0 == o.d0 && d1 == o.d1; }
};
bool same_size_axis(uint32_t n, std::vector<AxisClass>& cls) {
    cls.clear();
    const int32_t hi = (int32_t)n - 1;
    for (uint32_t x = 0; x < n; ++x) {
        const float u = ((float)x + 0.5f) / (float)n;
        const float t = fminf(fmaxf(u * (float)n - 0.5f, -1.0f), (float)n);
        const float f = floorf(t);
        const float fa = t - f;
        const int32_t x0 = std::min(std::max((int32_t)f, 0), hi), x1 = std::min(std::max((int32_t)f + 1, 0), hi);
        const AxisClass c{1.0f - fa, fa, x0 == (int32_t)x, x1 == (int32_t)x};
        if (!c.d0 && !c.d1) return false;
        if (std::find(cls.begin(), cls.end(), c) == cls.end()) cls.push_back(c);
    }
    return true;
}
uint8_t unorm8_ref(float a) {
    if (!(a > 0.0f)) return 0;
    if (a >= 1.0f) return 255;
    return (uint8_t)std::floor((double)a * 255.0 + 0.5);
}
// Every pixel of a same-size pass samples its own texel centre exactly (t == x): weights 1 and 0, the
// sample is the texel itself, before any quantisation (powers of two).
bool same_size_exact(uint32_t n) {
    for (uint32_t x = 0; x < n; ++x) {
        const float u = ((float)x + 0.5f) / (float)n;
        if (u * (float)n - 0.5f != (float)x) return false;
    }
    return true;
}
bool same_size_identity(uint32_t w, uint32_t h) {
    static thread_local std::vector<std::pair<uint64_t, bool>> memo;
    const uint64_t key = (uint64_t)w << 32 | h;
    for (const auto& m : memo)
        if (m.first == key) return m.second;
    std::vector<AxisClass> cx, cy;
    bool ok = same_size_axis(w, cx) && same_size_axis(h, cy);
    float lut[256];
    srgb_lut(lut);
    for (const AxisClass& X : cx)
        for (const AxisClass& Y : cy)
            for (int kind = 0; kind < 2 && ok; ++kind)
                for (int b = 0; b < 256 && ok; ++b) {
                    const float D = kind == 0 ? lut[b] : (float)b / 255.0f;
                    for (float O : {0.0f, 1.0f}) {
                        const float t00 = X.d0 && Y.d0 ? D : O, t10 = X.d1 && Y.d0 ? D : O;
                        const float t01 = X.d0 && Y.d1 ? D : O, t11 = X.d1 && Y.d1 ? D : O;
                        const float r = (t00 * X.ia + t10 * X.fa) * Y.ia + (t01 * X.ia + t11 * X.fa) * Y.fa;
                        if ((kind == 0 ? srgb_encode_ref(r) : unorm8_ref(r)) != b) ok = false;
                    }
                }
    if (memo.size() >= 16) memo.erase(memo.begin());
    memo.push_back({key, ok});
    return ok;
}

struct BloomPlan {
    uint32_t W, H, levels;
    uint32_t res[16][2];
};

// kawase_*sampling.rs:30-39: level l is (W, H) halved l times (integer), at least 1
BloomPlan bloom_plan(uint32_t W, uint32_t H, uint32_t levels) {
    BloomPlan p{W, H, levels, {}};
    uint32_t w = W, h = H;
    for (uint32_t l = 0; l < levels; ++l) {
        w = w ? w : 1u;
        h = h ? h : 1u;
        p.res[l][0] = w;
        p.res[l][1] = h;
        w /= 2u;
        h /= 2u;
    }
    return p;
}

// The separable plan of an up pass of this shape (bh_bloom_sep_plan), on the device, built at its first
// use and kept with the scratch set (64 B per column and row).  rx == 0: the same-size plan of the remixes
// (bh_bloom_same_plan, 8 B per column and row) followed by the list of its inexact columns, then rows (the
// fused epilogues' fix-up pixels).  Every plan is checked on the host before it is uploaded
// (bh_bloom_sep_verify / bh_bloom_same_verify: every block footprint inside its LDS tile, every read and
// index inside its tile and texture); a shape the builder refuses (texture sides above 65536) or whose
// check fails gets a plan with dev == nullptr, cached like the others, and its pass runs the general
// kernel -- with `dry_fail` (bh_bloom_check) a failed check is reported there instead.  In dry mode the
// plan stays on the host (dev points into `host`).  A capturing call never builds one (bh_bloom refuses a
// set not prepared outside capture).
// The column strips' storage limit per plan (3 words per strip column and row: 1.3 MB at 1920 x 1080)
constexpr size_t BH_STRIPS_BUDGET = (size_t)64 << 20;
// A plan the host check refused: in dry mode the check's failure; in a real bh_bloom a process-wide count and
// last message (bh_bloom_plan_failures) and one line on stderr, so that a regression in plan generation --
// bit-exact, but the slower general kernel -- does not pass silently.
std::atomic<uint64_t> g_plan_failures{0};
std::string g_plan_last;  // guarded by g_plan_mu
std::atomic_flag g_plan_mu = ATOMIC_FLAG_INIT;
void plan_failure(std::string* dry_fail, uint32_t ow, uint32_t oh, uint32_t tw, uint32_t th, uint32_t rx, uint32_t ry,
                  const std::string& why) {
    const std::string msg = "plan " + std::to_string(ow) + "x" + std::to_string(oh) + " <- " + std::to_string(tw) + "x" +
                            std::to_string(th) + " res " + std::to_string(rx) + "x" + std::to_string(ry) + ": " + why;
    if (dry_fail) {
        if (dry_fail->empty()) *dry_fail = msg;
        return;
    }
    while (g_plan_mu.test_and_set(std::memory_order_acquire)) std::this_thread::yield();
    g_plan_last = msg;
    g_plan_mu.clear(std::memory_order_release);
    if (g_plan_failures.fetch_add(1) == 0)
        std::fprintf(stderr, "bh_bloom: a host check refused a plan; its pass runs the general kernel (same bytes, "
                             "slower): %s\n", msg.c_str());
}
// Returned by value: the cache is a vector that later plans reallocate.  (Round 4's memory-access fault:
// a pointer into it, held across the next call, read a freed record's fix-up counts)
bh_ctx::SepPlan sep_plan(bh_ctx::BloomScratch* b, bool capturing, std::string* dry_fail, uint32_t ow, uint32_t oh,
                         uint32_t tw, uint32_t th, uint32_t rx, uint32_t ry, int* err, uint32_t org = 0, bool fix = false) {
    const std::array<uint32_t, 8> key{ow, oh, tw, th, rx, ry, org, fix ? 1u : 0u};
    for (const auto& p : b->sep_plans)
        if (p.key == key) return p;
    bh_ctx::SepPlan P;
    P.key = key;
    if (capturing) {
        *err = (int)hipErrorStreamCaptureUnsupported;
        return P;
    }
    auto h = std::make_shared<std::vector<uint32_t>>();
    std::string why;
    bool ok;
    if (rx) {
        h->resize(32u * ((size_t)ow + oh));
        P.ext = bh_bloom_sep_plan(ow, oh, tw, th, rx, ry, h->data(), org);
        ok = P.ext >= 0 && bh_bloom_sep_verify(ow, oh, tw, th, rx, ry, h->data(), P.ext, org, fix, &why);
    } else {
        h->resize(2u * ((size_t)ow + oh));
        ok = bh_bloom_same_plan(ow, oh, h->data());
        if (ok) {
            std::vector<uint32_t> cols, rows;
            for (uint32_t x = 0; x < ow; ++x)
                if ((*h)[2u * x + 1u] != 0u) cols.push_back(x);
            for (uint32_t y = 0; y < oh; ++y)
                if ((*h)[2u * ((size_t)ow + y) + 1u] != 0u) rows.push_back(y);
            P.nc = (uint32_t)cols.size();
            P.nr = (uint32_t)rows.size();
            h->insert(h->end(), cols.begin(), cols.end());
            h->insert(h->end(), rows.begin(), rows.end());
            ok = bh_bloom_same_verify(ow, oh, h->data(), P.nc, P.nr, &why);
            if (ok) {  // the in-block fix's grid origin and residual list (checked where the fix-up launches)
                std::vector<uint32_t> rc, rr, rc2, rr2;
                P.org = bh_bloom_same_org(ow, oh, h->data(), &rc, &rr, &rc2, &rr2);
                P.nrc = (uint32_t)rc.size();
                P.nrr = (uint32_t)rr.size();
                P.nrc2 = (uint32_t)rc2.size();
                P.nrr2 = (uint32_t)rr2.size();
                for (const auto* v : {&rc, &rr, &rc2, &rr2}) h->insert(h->end(), v->begin(), v->end());
                // the three lists' records, 16-byte aligned (the kernel reads them as uint4)
                const size_t lists = 2u * ((size_t)ow + oh), n_all = P.nc + P.nr + P.nrc + P.nrr + P.nrc2 + P.nrr2;
                h->resize((h->size() + 3u) & ~(size_t)3u, 0u);
                P.rec = h->size();
                h->resize(P.rec + 8u * n_all, 0u);
                uint32_t* R = h->data() + P.rec;
                const uint32_t* L = h->data() + lists;
                bh_bloom_fixup_records(ow, oh, h->data(), L, P.nc, P.nr, R);
                L += P.nc + P.nr; R += 8u * (P.nc + P.nr);
                bh_bloom_fixup_records(ow, oh, h->data(), L, P.nrc, P.nrr, R);
                L += P.nrc + P.nrr; R += 8u * (P.nrc + P.nrr);
                bh_bloom_fixup_records(ow, oh, h->data(), L, P.nrc2, P.nrr2, R);
                // every list's records as the fix-up kernels read them (a failure drops the plan)
                {
                    const uint32_t* Lc = h->data() + lists;
                    const uint32_t* Rc = h->data() + P.rec;
                    const uint32_t nlist[3][2] = {{P.nc, P.nr}, {P.nrc, P.nrr}, {P.nrc2, P.nrr2}};
                    for (int li = 0; ok && li < 3; ++li) {
                        ok = bh_bloom_records_verify(ow, oh, h->data(), Lc, nlist[li][0], nlist[li][1], Rc, nullptr, 0u, &why);
                        Lc += nlist[li][0] + nlist[li][1];
                        Rc += 8u * (nlist[li][0] + nlist[li][1]);
                    }
                }
                // the column strips of the final fix-up (BH_BLOOM_NO_STRIPS: off, A/B), within a storage budget
                static const bool no_strips = std::getenv("BH_BLOOM_NO_STRIPS") != nullptr;
                if (ok && !no_strips && P.nc > 0u) {
                    const size_t at = h->size();
                    h->resize(at + ow, 0u);
                    const uint32_t stw = bh_bloom_strip_table(ow, h->data() + lists, P.nc, h->data() + at);
                    if (stw > 0u && 3u * (size_t)stw * oh * 4u <= BH_STRIPS_BUDGET) {
                        // word 7 of each column record: 1 + the column's strip column
                        for (uint32_t k = 0; k < P.nc; ++k) (*h)[P.rec + 8u * k + 7u] = (*h)[at + (*h)[lists + k]];
                        // checked before upload: the gather kernel clamps its strip column, so a wrong table would
                        // give wrong pixels, not a fault; a failing table drops the strips (the plain fix-up runs)
                        std::string swhy;
                        if (bh_bloom_records_verify(ow, oh, h->data(), h->data() + lists, P.nc, 0u, h->data() + P.rec,
                                                    h->data() + at, stw, &swhy)) {
                            P.stc = at;
                            P.stw = stw;
                        } else {
                            for (uint32_t k = 0; k < P.nc; ++k) (*h)[P.rec + 8u * k + 7u] = 0u;
                            h->resize(at);
                            plan_failure(dry_fail, ow, oh, tw, th, rx, ry, "strips dropped: " + swhy);
                        }
                    } else {
                        h->resize(at);
                    }
                }
            }
        }
    }
    if (!ok) {
        if (!why.empty()) plan_failure(dry_fail, ow, oh, tw, th, rx, ry, why);
        bh_ctx::SepPlan none;
        none.key = key;
        b->sep_plans.push_back(none);
        return none;
    }
    if (dry_fail) {
        P.host = h;
        P.dev = h->data();
    } else {
        hipError_t e = hipMalloc(&P.dev, h->size() * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMemcpy(P.dev, h->data(), h->size() * sizeof(uint32_t), hipMemcpyHostToDevice);
        if (e == hipSuccess && P.stc) e = hipMalloc(&P.strips, 3u * (size_t)P.stw * oh * 4u);
        if (e != hipSuccess) {
            if (P.dev) (void)hipFree(P.dev);
            if (P.strips) (void)hipFree(P.strips);
            *err = (int)e;
            bh_ctx::SepPlan none;
            none.key = key;
            return none;
        }
    }
    b->sep_plans.push_back(P);
    return P;
}

struct BloomRun {
    bh_ctx* c;
    bh_ctx::BloomScratch* B;
    bool capturing;
    hipStream_t s;
    std::string* dry_fail;  // bh_bloom_check's dry mode: plans on the host, launches checked, not launched
    int err = 0;
    void pass(uint32_t sh, const uint32_t* a, uint32_t aw, uint32_t ah, const uint32_t* b, const uint32_t* res,
              uint32_t* out, uint32_t ow, uint32_t oh) {
        if (err != 0) return;
        bh_ctx::SepPlan sp{};
        if (sh == bh_bloom_shader_up && bh_bloom_up_uses_sep(ow, oh, aw, ah, res[0], res[1]))
            sp = sep_plan(B, capturing, dry_fail, ow, oh, aw, ah, res[0], res[1], &err);
        if (err == 0)
            err = bh_launch_bloom_pass(sh, c->lut, c->enc, c->enc_b, c->enc_e, a, aw, ah, b, res[0], res[1], out, ow, oh,
                                       sp.dev, sp.ext, s);
    }
    // the fused chains' blur downsamples src (res[0]) -> down[1] -> ... -> down[levels - 1]; returns the
    // last level.  An intermediate level is read by nothing but the next downsample, so pairs run as one
    // pass (bh_launch_bloom_down2, the intermediate not stored); BH_BLOOM_NO_DOWN2 runs them one by one (A/B)
    // first = 3: the Y pass already wrote down[2] (bh_launch_bloom_y's fused down2)
    const uint32_t* downs(const uint32_t* src, uint32_t levels, uint32_t** down, const BloomPlan& P, uint32_t first = 1) {
        static const bool no_down2 = std::getenv("BH_BLOOM_NO_DOWN2") != nullptr;
        const uint32_t* dn = first == 3 ? down[2] : src;
        uint32_t l = first;
        for (; !no_down2 && l + 1 < levels && err == 0; l += 2) {
            err = bh_launch_bloom_down2(c->lut, c->enc, c->enc_b, c->enc_e, dn, P.res[l - 1][0], P.res[l - 1][1],
                                        P.res[l][0], P.res[l][1], down[l + 1], P.res[l + 1][0], P.res[l + 1][1], s);
            dn = down[l + 1];
        }
        for (; l < levels; ++l) {
            pass(bh_bloom_shader_down, dn, P.res[l - 1][0], P.res[l - 1][1], nullptr, P.res[l - 1], down[l], P.res[l][0],
                 P.res[l][1]);
            dn = down[l];
        }
        return dn;
    }
};

// bh_bloom's chain on scratch set B: the reference's passes one by one (literal) or the fused forms.
// dry_fail (bh_bloom_check): the plans stay on the host and the launchers check their launch instead of
// launching (bh_bloom.hip dry mode); the scratch pointers are then placeholders that nothing dereferences.
int bloom_chain(bh_ctx* c, bh_ctx::BloomScratch* B, bool capturing, std::string* dry_fail, const void* col,
                const void* blackout, uint32_t W, uint32_t H, uint32_t levels, uint32_t schedule, void* out,
                hipStream_t s) {
    const BloomPlan P = bloom_plan(W, H, levels);
    // AUTO: the fused chain when every same-size sample is exact (powers of two); else the general fused chain
    // (the remixes sample through the same-size plan; the same-size copies vanish where they are proven identities
    // on stored texels, same_size_identity, and run as same-size copy passes where not: 3840x2160, 3440x1440,
    // ...); the literal pass list when a plan is refused (or BH_BLOOM_NO_GENERAL_COPIES and a copy is not an
    // identity: the round-5 rule, A/B)
    const uint32_t wl = P.res[levels - 1][0], hl = P.res[levels - 1][1];
    const bool fused = schedule == BH_BLOOM_AUTO && same_size_exact(W) && same_size_exact(H) && same_size_exact(wl) &&
                       same_size_exact(hl);
    const bool id_full = same_size_identity(W, H), id_low = same_size_identity(wl, hl);
    static const bool no_copies = std::getenv("BH_BLOOM_NO_GENERAL_COPIES") != nullptr;
    const bool general = schedule == BH_BLOOM_AUTO && !fused && (!no_copies || (id_full && id_low));
    bh_ctx::SepPlan same;
    uint32_t** T = B->tex.data();
    uint32_t **copy_in = T, **remix_in0 = T + levels, **remix_in1 = T + 2 * levels;
    uint32_t* blur_in = T[3 * levels];
    uint32_t* final_in1 = T[3 * levels + 1];
    uint32_t **down = T + 3 * levels + 2, **up = T + 4 * levels + 2;
    const uint32_t* X = (const uint32_t*)blackout;
    const uint32_t* C = (const uint32_t*)col;
    uint32_t* O = (uint32_t*)out;
    const uint32_t full[2] = {W, H};
    BloomRun R{c, B, capturing, s, dry_fail};
    const uint32_t L = levels - 1;
    if (fused) {
        // same-size passes are identities (same_size_identity): see bh_bloom.hip
        const uint32_t* S = X;
        bool d2 = false;  // the Y pass also wrote the blur's first two downsamples (down[2])
        if (levels > 1) {
            if (R.err == 0)
                R.err = bh_launch_bloom_y(c->lut, c->enc, c->enc_b, c->enc_e, X, copy_in[1], W, H,
                                          levels >= 3 ? down[2] : nullptr, &d2, s);
            S = copy_in[1];
        }
        // down[0] == S; up[levels-1] == down[levels-1]
        const uint32_t* u_src = R.downs(S, levels, down, P, d2 ? 3u : 1u);
        for (uint32_t l = 0; l + 1 < levels; ++l) {
            const uint32_t ti = levels - l - 2;
            R.pass(bh_bloom_shader_up, u_src, P.res[ti + 1][0], P.res[ti + 1][1], nullptr, P.res[l], up[ti],
                   P.res[ti][0], P.res[ti][1]);
            u_src = up[ti];
        }
        if (R.err == 0)
            R.err = bh_launch_bloom_final(c->lut, c->enc, c->enc_b, c->enc_e, C, S, u_src, P.res[L][0], P.res[L][1], O, W, H, s);
    } else if (general && (same = sep_plan(B, capturing, dry_fail, W, H, W, H, 0u, 0u, &R.err), same.dev != nullptr)) {
        // general fused chain (same-size passes are identities, same_size_identity): U1 = up(X) at full
        // size, Y = remix(X, U1) through the same-size plan, the blur's downsamples and upsamples from Y,
        // B = its last up pass, out = remix(col, q(remix(Y, B))) through the plan.  The two full-size
        // up passes with a separable plan carry the remixes as epilogues for the pixels whose column and
        // row sample exactly (bh_bloom.hip up_sep_kernel, EPI_Y / EPI_FINAL) and a fix-up pass covers the
        // inexact columns and rows; other plans run the plain pass and the plan remix kernels.
        const uint32_t* plan = same.dev;
        const uint32_t* list = plan ? plan + 2u * ((size_t)W + H) : nullptr;
        const uint32_t* residual = list ? list + same.nc + same.nr : nullptr;
        const uint32_t* residual2 = residual ? residual + same.nrc + same.nrr : nullptr;
        // The final epilogue's in-block fix (FIX2) only with BH_BLOOM_FIX2 -- measured slower than its fix-up pass
        // (1920x1080 0.1237 -> 0.1256 ms: three block barriers in the chain's longest-lived waves;
        // profiles/r05/bloom_fix2/)
        static const bool fix2 = std::getenv("BH_BLOOM_FIX2") != nullptr;
        // an up pass at full size into `aux` with epilogue `epi` (own0, own1 its own-texel inputs), then the
        // fix-up of the inexact pixels -- or the plain pass and the remix kernel
        auto fused_up = [&](uint32_t epi, const uint32_t* src, uint32_t sw, uint32_t sh, const uint32_t* res,
                            uint32_t* aux, const uint32_t* own0, const uint32_t* own1, uint32_t* dst) {
            if (R.err != 0) return;
            bh_ctx::SepPlan sp{};
            // the epilogues' in-block fixes (quad kernel: the grid at the same-size plan's origin, the fix-up pass
            // over the residual list only): the Y epilogue's was removed in round 6 -- it gave wrong bytes at frame
            // sizes outside the test list (a seeded random-size sweep: e.g. 1846x1392, 177x1706) --, the final
            // epilogue's (BH_BLOOM_FIX2) is an A/B arm; otherwise the fix-up pass covers every inexact column and row
            const bool fix = epi == 2u && fix2;
            const uint32_t org = fix ? same.org : 0u;
            if (bh_bloom_up_uses_sep(W, H, sw, sh, res[0], res[1]))
                sp = sep_plan(B, capturing, dry_fail, W, H, sw, sh, res[0], res[1], &R.err, org, fix);
            if (R.err != 0) return;
            // the final epilogue writes the column strips its fix-up reads (bh_bloom.hip STRIPS)
            const uint32_t* stc = epi == 2u && same.stc ? plan + same.stc : nullptr;
            bool strips = false;
            if (sp.dev && bh_launch_bloom_sep(c->lut, c->enc, c->enc_b, c->enc_e, src, sw, sh, res[0], res[1], sp.dev,
                                              sp.ext, epi, own0, own1, plan, dst, aux, W, H, org, fix, stc, same.strips,
                                              same.stw, &strips, s) == 0) {
                const bool fixed = fix && bh_bloom_sep_fix_ok(sp.ext, W, H, epi);
                const uint32_t* rl = epi == 1u ? residual : residual2;
                const uint32_t rc = epi == 1u ? same.nrc : same.nrc2, rr = epi == 1u ? same.nrr : same.nrr2;
                // the list's records: full, residual 1, residual 2 in that order after same.rec
                const size_t rk = !fixed ? 0u : epi == 1u ? same.nc + same.nr : same.nc + same.nr + same.nrc + same.nrr;
                const uint32_t* recs = same.rec ? plan + same.rec + 8u * rk : nullptr;
                R.err = bh_launch_bloom_fixup(c->lut, c->enc, c->enc_b, c->enc_e, epi, own0, epi == 1u ? aux : own1, aux,
                                              plan, fixed ? rl : list, fixed ? rc : same.nc, fixed ? rr : same.nr, dst, W, H,
                                              fixed ? (int32_t)same.org : -1, recs, strips && !fixed ? stc : nullptr,
                                              same.strips, same.stw, s);
                return;
            }
            R.pass(bh_bloom_shader_up, src, sw, sh, nullptr, res, aux, W, H);
            if (R.err != 0) return;
            R.err = epi == 1u ? bh_launch_bloom_remix_plan(c->lut, c->enc, c->enc_b, c->enc_e, own0, aux, plan, dst, W, H, s)
                              : bh_launch_bloom_remix2_plan(c->lut, c->enc, c->enc_b, c->enc_e, own0, own1, aux, plan, dst,
                                                            W, H, s);
        };
        // A copy that is not an identity (same_size_identity) runs as the literal chain's pass: X1 = copy(X) (the
        // first loop's down[0] and remix_in0[0]), X2 = its same-size down (the blur of one level), S1 = copy(Y)
        // (the last blur's down[0] and remix_in0[L]), and the same-size down at the blur's smallest level.
        const uint32_t* S = X;  // levels 1: the loop never runs, the blur reads X itself
        if (levels > 1) {
            const uint32_t *X1 = X, *X2 = X;
            if (!id_full) {  // same_copy_kernel, twice
                if (R.err == 0)
                    R.err = bh_launch_bloom_same_copy(c->lut, c->enc, c->enc_b, c->enc_e, X, plan, remix_in0[0], W, H, s);
                if (R.err == 0)
                    R.err = bh_launch_bloom_same_copy(c->lut, c->enc, c->enc_b, c->enc_e, remix_in0[0], plan, blur_in, W, H, s);
                X1 = remix_in0[0];
                X2 = blur_in;
            }
            fused_up(1u, X2, W, H, full, remix_in1[0], X1, nullptr, copy_in[1]);
            S = copy_in[1];
        }
        if (!id_full) {
            if (R.err == 0)
                R.err = bh_launch_bloom_same_copy(c->lut, c->enc, c->enc_b, c->enc_e, S, plan, remix_in0[L], W, H, s);
            S = remix_in0[L];
        }
        const uint32_t* u_src = R.downs(S, levels, down, P);
        if (!id_low) {
            R.pass(bh_bloom_shader_down, u_src, wl, hl, nullptr, P.res[L], up[L], wl, hl);
            u_src = up[L];
        }
        for (uint32_t l = 0; l + 1 < levels; ++l) {
            const uint32_t ti = levels - l - 2;
            R.pass(bh_bloom_shader_up, u_src, P.res[ti + 1][0], P.res[ti + 1][1], nullptr, P.res[l], up[ti],
                   P.res[ti][0], P.res[ti][1]);
            u_src = up[ti];
        }
        const uint32_t uw = levels > 1 ? P.res[0][0] : W, uh = levels > 1 ? P.res[0][1] : H;  // up[0] is W x H
        fused_up(2u, u_src, uw, uh, P.res[L], remix_in1[L], C, S, O);
    } else if (R.err == 0) {
        // literal: the reference's render passes in order (also the general chain's fallback when the host
        // refuses its same-size plan) (oracle/bh_bloom_oracle.c, bho_bloom)
        hipError_t e;
        if (!dry_fail && (e = hipMemcpyAsync(copy_in[0], X, (size_t)W * H * 4u, hipMemcpyDeviceToDevice, s)) != hipSuccess)
            return hip_fail(e, "hipMemcpyAsync(bloom)");
        auto blur = [&](uint32_t lv, uint32_t* dst) {
            // blurs[k] with `lv` levels; its input (down[0]) was written by the copy pass
            for (uint32_t l = 1; l < lv; ++l)
                R.pass(bh_bloom_shader_down, down[l - 1], P.res[l - 1][0], P.res[l - 1][1], nullptr, P.res[l - 1],
                       down[l], P.res[l][0], P.res[l][1]);
            R.pass(bh_bloom_shader_down, down[lv - 1], P.res[lv - 1][0], P.res[lv - 1][1], nullptr, P.res[lv - 1],
                   up[lv - 1], P.res[lv - 1][0], P.res[lv - 1][1]);
            for (uint32_t l = 0; l + 1 < lv; ++l)
                R.pass(bh_bloom_shader_up, up[lv - l - 1], P.res[lv - l - 1][0], P.res[lv - l - 1][1], nullptr, P.res[l],
                       up[lv - l - 2], P.res[lv - l - 2][0], P.res[lv - l - 2][1]);
            R.pass(bh_bloom_shader_up, up[0], W, H, nullptr, P.res[lv - 1], dst, W, H);
        };
        for (uint32_t level = 0; level + 1 < levels; ++level) {
            R.pass(bh_bloom_shader_copy, copy_in[0], W, H, nullptr, full, down[0], W, H);
            R.pass(bh_bloom_shader_copy, copy_in[0], W, H, nullptr, full, remix_in0[0], W, H);
            blur(1, remix_in1[0]);
            R.pass(bh_bloom_shader_remix, remix_in0[0], W, H, remix_in1[0], full, copy_in[level + 1], W, H);
        }
        R.pass(bh_bloom_shader_copy, copy_in[L], W, H, nullptr, full, down[0], W, H);
        R.pass(bh_bloom_shader_copy, copy_in[L], W, H, nullptr, full, remix_in0[L], W, H);
        blur(levels, remix_in1[L]);
        R.pass(bh_bloom_shader_remix, remix_in0[L], W, H, remix_in1[L], full, final_in1, W, H);
        R.pass(bh_bloom_shader_remix, C, W, H, final_in1, full, O, W, H);
        (void)blur_in;
    }
    if (R.err != 0) return hip_fail((hipError_t)R.err, "bloom launch");
    return BH_OK;
}
}  // namespace

extern "C" {

int bh_bloom(bh_ctx* c, const void* col, const void* blackout, uint32_t W, uint32_t H, uint32_t levels,
             uint32_t schedule, void* out, void* stream) {
    // W, H <= 65536 as bh_render: the bloom kernels index texels with 32 bits (y * w + x < 2^32)
    if (!c || !col || !blackout || !out || W == 0 || H == 0 || W > 65536u || H > 65536u || levels < 1 || levels > 12 ||
        schedule > BH_BLOOM_LITERAL)
        return bad_arg(__func__, __LINE__);
    hipError_t e;
    DeviceScope dev(c->device);
    if (dev.err != hipSuccess) return hip_fail(dev.err, "hipSetDevice");
    hipStream_t s = (hipStream_t)stream;
    const BloomPlan P = bloom_plan(W, H, levels);
    // scratch: [0, 3*levels) copy_in / remix_in0 / remix_in1 (full), then blur_in, final_in1 (full),
    // then down[levels], up[levels] at res[l]
    const uint64_t key = ((uint64_t)W << 40) ^ ((uint64_t)H << 16) ^ levels;
    const bool capturing = stream_capturing(s);
    bh_ctx::BloomScratch* B = nullptr;
    for (auto& b : c->blooms)
        if (b.key == key) B = &b;
    if (capturing) {
        // graph contract: nothing is allocated or uploaded under capture, and a set a graph uses is kept
        if (!B || !(B->prepared & (1u << schedule))) {
            g_last_error = "bh_bloom: the first call of a (size, levels, schedule) allocates; run it once before "
                           "capturing it into a graph";
            return BH_ERR_UNSUPPORTED;
        }
        B->captured = true;
    }
    if (!B) {
        bh_ctx::BloomScratch n;
        n.key = key;
        auto alloc = [&](size_t bytes) {
            uint32_t* t = nullptr;
            if ((e = hipMalloc(&t, bytes)) == hipSuccess) n.tex.push_back(t);
            return e == hipSuccess;
        };
        bool ok = true;
        for (uint32_t i = 0; ok && i < 3u * levels + 2u; ++i) ok = alloc((size_t)W * H * 4u);
        for (uint32_t k = 0; ok && k < 2; ++k)
            for (uint32_t l = 0; ok && l < levels; ++l) ok = alloc((size_t)P.res[l][0] * P.res[l][1] * 4u);
        if (!ok) {
            free_bloom_scratch(n);
            return e == hipErrorOutOfMemory ? BH_ERR_OUT_OF_MEMORY : hip_fail(e, "hipMalloc(bloom)");
        }
        if (c->blooms.size() >= BH_BLOOM_SETS) {  // evict the least recently used set no graph holds
            size_t v = c->blooms.size();
            for (size_t i = 0; i < c->blooms.size(); ++i)
                if (!c->blooms[i].captured && (v == c->blooms.size() || c->blooms[i].last_use < c->blooms[v].last_use))
                    v = i;
            if (v < c->blooms.size()) {
                free_bloom_scratch(c->blooms[v]);
                c->blooms.erase(c->blooms.begin() + (long)v);
            }
        }
        c->blooms.push_back(std::move(n));
        B = &c->blooms.back();
    }
    B->last_use = ++c->bloom_clock;
    const int st = bloom_chain(c, B, capturing, nullptr, col, blackout, W, H, levels, schedule, out, s);
    if (st != BH_OK) return st;
    if (!capturing) B->prepared |= 1u << schedule;
    return BH_OK;
}

int bh_bloom_check(uint32_t W, uint32_t H, uint32_t levels, uint32_t schedule, uint64_t* out_launches, char* out_plan,
                   size_t plan_len) {
    if (W == 0 || H == 0 || W > 65536u || H > 65536u || levels < 1 || levels > 12 || schedule > BH_BLOOM_LITERAL)
        return bad_arg(__func__, __LINE__);
    bh_ctx c;  // no device: nothing below allocates, uploads or launches
    bh_ctx::BloomScratch B;
    for (uint32_t i = 0; i < 5u * levels + 2u; ++i) B.tex.push_back(reinterpret_cast<uint32_t*>((uintptr_t)(i + 1u) << 20));
    const void* in = reinterpret_cast<const void*>((uintptr_t)1 << 40);
    std::string fail, dfail, plan;
    uint64_t launches = 0, checks = 0;
    bh_bloom_dry_begin();
    const int st = bloom_chain(&c, &B, false, &fail, in, in, W, H, levels, schedule, const_cast<void*>(in), nullptr);
    const bool ok = bh_bloom_dry_end(&launches, &checks, &dfail, &plan);
    if (out_launches) *out_launches = launches;
    if (out_plan && plan_len) {
        const size_t n = std::min(plan.size(), plan_len - 1);
        std::memcpy(out_plan, plan.data(), n);
        out_plan[n] = '\0';
    }
    if (!ok || !fail.empty() || st != BH_OK) {
        g_last_error = "bh_bloom_check " + std::to_string(W) + "x" + std::to_string(H) + " levels " +
                       std::to_string(levels) + ": " + (!dfail.empty() ? dfail : !fail.empty() ? fail : g_last_error);
        return BH_ERR_INTERNAL;
    }
    return BH_OK;
}

int64_t bh_bloom_plan_failures(char* out_last, size_t len) {
    if (out_last && len) {
        while (g_plan_mu.test_and_set(std::memory_order_acquire)) std::this_thread::yield();
        const size_t n = std::min(g_plan_last.size(), len - 1);
        std::memcpy(out_last, g_plan_last.data(), n);
        out_last[n] = '\0';
        g_plan_mu.clear(std::memory_order_release);
    }
    return (int64_t)g_plan_failures.load();
}

int bh_graph_release(bh_ctx* c) {
    if (!c) return bad_arg(__func__, __LINE__);
    for (auto& o : c->orders) o.captured = false;
    for (auto& b : c->blooms) b.captured = false;
    return BH_OK;
}

int64_t bh_shard_tile_count(uint32_t width, uint32_t height, uint32_t shard_index, uint32_t shard_count) {
    if (width == 0 || height == 0 || shard_count == 0 || shard_index >= shard_count) return bad_arg(__func__, __LINE__);
    return (int64_t)bh::shard_tile_count((width + 7u) / 8u, (height + 7u) / 8u, shard_index, shard_count);
}

// Which build of the exact kernels runs a launch (BH_SCHED_FLAG_ISSUE_ORDER / _LATENCY force one).  The
// source-order build issues the bulk of the steps faster; the machine-scheduled one, whose tail loop
// also runs the packed step, marches a lone wave's serial chain faster.  A launch is throughput-bound
// when its tiles in flight (all frames') outlast the capped rays' chains: about 384 tiles per CU at
// cap 512 (the bulk runs ~1.2 us per tile and CU, a cap-512 chain ~0.45 ms), scaled by the cap.
// Measured (A/B r02, profiles/r02/variants.log, ms per frame, source-order / scheduled): 4096x2048
// cap 512 one frame (512 tiles/CU) 0.644 / 0.687; its 1/8 shard 0.445 / 0.363; 8192x4096's 1/8 shard
// 0.61 / 0.39; cap 1000 camera C 0.957 / 0.737; 1920x1080 cap 256 0.253 / 0.205; in 8-frame launches
// cap 1000 0.669 / 0.698, 1920x1080 0.165 / 0.171, 8192x4096's 1/8 shard 0.322 / 0.337.
static bool march_variant_issue_order(const bh_render_desc* d, uint32_t n_tiles, uint32_t n_frames, uint32_t cus) {
    if (d->schedule & BH_SCHED_FLAG_ISSUE_ORDER) return true;
    if (d->schedule & BH_SCHED_FLAG_LATENCY) return false;
    const uint64_t tiles = (uint64_t)n_tiles * n_frames;
    return tiles * 512ull >= 384ull * (cus ? cus : 256u) * d->max_iters;
}

static void free_frame_table(bh_ctx::FrameTable& t) {
    for (uint32_t k = 0; k < bh_ctx::FRAME_RING; ++k) {
        if (t.done[k]) { (void)hipEventSynchronize(t.done[k]); (void)hipEventDestroy(t.done[k]); }
        if (t.host[k]) (void)hipHostFree(t.host[k]);
    }
    if (t.dev) (void)hipFree(t.dev);
    t = bh_ctx::FrameTable{};
}

// Stage the n frames' arguments in the device table of stream s (created at its first use): a pinned
// ring slot is filled once its previous copy has executed, then copied in on the stream, ahead of the
// order and march kernels that read it.  *dev receives the table.
static int stage_frame_table(bh_ctx* c, hipStream_t s, const bh::FrameArgs* frames, uint32_t n,
                             const bh::FrameArgs** dev) {
    if (stream_capturing(s)) {
        g_last_error = "bh_render_frames: more than 32 frames per call cannot be captured into a graph";
        return BH_ERR_UNSUPPORTED;
    }
    bh_ctx::FrameTable* t = nullptr;
    for (auto& x : c->frame_tables)
        if (x.stream == (void*)s) t = &x;
    if (!t) {
        bh_ctx::FrameTable n_t;
        n_t.stream = (void*)s;
        const size_t bytes = sizeof(bh::FrameArgs) * BH_MAX_FRAMES;
        hipError_t he = hipMalloc(&n_t.dev, bytes);
        for (uint32_t k = 0; he == hipSuccess && k < bh_ctx::FRAME_RING; ++k) {
            he = hipHostMalloc(&n_t.host[k], bytes, hipHostMallocDefault);
            if (he == hipSuccess) he = hipEventCreateWithFlags(&n_t.done[k], hipEventDisableTiming);
        }
        if (he != hipSuccess) {
            free_frame_table(n_t);
            return he == hipErrorOutOfMemory ? BH_ERR_OUT_OF_MEMORY : hip_fail(he, "frame table");
        }
        c->frame_tables.push_back(n_t);
        t = &c->frame_tables.back();
    }
    *dev = t->dev;
    // the same frames as the stream's previous table (a re-rendered camera path): nothing to copy,
    // the stream's earlier copy precedes this launch
    if (t->last.size() == n && std::memcmp(t->last.data(), frames, sizeof(bh::FrameArgs) * n) == 0) return BH_OK;
    const uint32_t k = t->next;
    t->next = (k + 1u) % bh_ctx::FRAME_RING;
    hipError_t he = hipEventSynchronize(t->done[k]);  // a never-recorded event is complete
    if (he == hipSuccess) {
        std::memcpy(t->host[k], frames, sizeof(bh::FrameArgs) * n);
        he = hipMemcpyAsync(t->dev, t->host[k], sizeof(bh::FrameArgs) * n, hipMemcpyHostToDevice, s);
    }
    if (he == hipSuccess) he = hipEventRecord(t->done[k], s);
    if (he != hipSuccess) {
        t->last.clear();
        return hip_fail(he, "frame table upload");
    }
    t->last.assign(frames, frames + n);
    return BH_OK;
}

// The temporal-order state of (geometry, shard, stream): found, or created (allocating; the LRU state
// is evicted beyond BH_ORDER_STATES).  New states start with all costs 0 and an empty histogram.
// Graph contract (include/bh_render.h): a state used by a launch captured into a graph is marked and
// never evicted (its buffers are what the graph's kernels read and write); when every state is marked
// the ctx keeps more than BH_ORDER_STATES instead of evicting one.  A capturing stream cannot create a
// state (the allocation and the reset are not capturable work): BH_ERR_UNSUPPORTED.
static int order_state(bh_ctx* c, const bh_render_desc* d, uint64_t nt, hipStream_t s, bool capturing,
                       bh_ctx::OrderState** out) {
    const uint64_t pser = d->partition ? d->partition->serial : 0u;
    for (auto& o : c->orders)
        if (o.width == d->width && o.height == d->height && o.shard_index == d->shard_index &&
            o.shard_count == d->shard_count && o.partition == pser && o.n_tiles == nt && o.stream == (void*)s) {
            o.last_use = ++c->order_clock;
            if (capturing) {
                if (!o.valid) {
                    g_last_error = "bh_render: this (geometry, shard, stream) must be rendered once outside graph capture";
                    return BH_ERR_UNSUPPORTED;
                }
                o.captured = true;
            }
            *out = &o;
            return BH_OK;
        }
    if (capturing) {
        g_last_error = "bh_render: the first render of a (geometry, shard, stream) allocates; render it once "
                       "before capturing it into a graph";
        return BH_ERR_UNSUPPORTED;
    }
    bh_ctx::OrderState n;
    n.width = d->width; n.height = d->height; n.shard_index = d->shard_index; n.shard_count = d->shard_count;
    n.partition = pser;
    n.n_tiles = nt;
    n.stream = (void*)s;
    const size_t cw = bh::ORDER_WORDS * sizeof(uint32_t);
    hipError_t he;
    if ((he = hipMalloc(&n.tile_cost, nt)) != hipSuccess || (he = hipMalloc(&n.order, nt * sizeof(uint32_t))) != hipSuccess ||
        (he = hipMalloc(&n.counters, cw)) != hipSuccess) {
        if (n.tile_cost) (void)hipFree(n.tile_cost);
        if (n.order) (void)hipFree(n.order);
        return he == hipErrorOutOfMemory ? BH_ERR_OUT_OF_MEMORY : hip_fail(he, "hipMalloc(temporal order)");
    }
    if (c->orders.size() >= BH_ORDER_STATES) {  // evict the least recently used state no graph holds
        size_t v = c->orders.size();
        for (size_t i = 0; i < c->orders.size(); ++i)
            if (!c->orders[i].captured && (v == c->orders.size() || c->orders[i].last_use < c->orders[v].last_use)) v = i;
        if (v < c->orders.size()) {
            auto& o = c->orders[v];
            (void)hipFree(o.tile_cost); (void)hipFree(o.order); (void)hipFree(o.counters);
            c->orders.erase(c->orders.begin() + (long)v);
        }
    }
    n.last_use = ++c->order_clock;
    c->orders.push_back(n);
    *out = &c->orders.back();
    return BH_OK;
}

// Per-frame invariants with the oracle's op sequence (correctly rounded f32, no contraction):
// c_ps = ((-normalize(ro0)) * 1.5) * RS (src/black_hole_maybe.wgsl:294).
static void frame_args(const bh_camera_uniform* cam, float rs, const bh_render_desc* d, bh::FrameArgs* F) {
    for (int k = 0; k < 3; ++k) {
        F->pos[k] = cam->pos[k];
        F->c0[k] = cam->world_tri[0][k];
        F->c1[k] = cam->world_tri[1][k];
        F->c2[k] = cam->world_tri[2][k];
    }
    const float x = F->pos[0], y = F->pos[1], z = F->pos[2];
    const float len = std::sqrt((x * x + y * y) + z * z);
    const float n[3] = {x / len, y / len, z / len};
    for (int k = 0; k < 3; ++k) F->cps[k] = (-n[k] * 1.5f) * rs;
    F->out_col = d->out_col; F->out_blackout = d->out_blackout;
    F->dbg_n_rk = d->dbg_n_rk; F->dbg_fate = d->dbg_fate; F->dbg_steps = d->dbg_steps;
}

// What a frame's per-tile costs (the march's step counts) depend on: the camera, the shader uniforms and the
// launch shape -- FNV-1a over those fields' bits (padding and the unused bg_brightness left out).  The
// outputs, their format and the sky do not change a step count.
static uint64_t frame_cost_key(const bh_camera_uniform* cam, const bh_uniforms* U, const bh_render_desc* d) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) {
        const unsigned char* b = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    };
    mix(cam->pos, sizeof(float) * 3);
    for (int k = 0; k < 3; ++k) mix(cam->world_tri[k], sizeof(float) * 3);
    for (int k = 0; k < 3; ++k) mix(cam->screen_tri[k], sizeof(float) * 3);
    mix(&U->rs, 4); mix(&U->delta_time_mult, 4); mix(&U->blackout_eh, 4); mix(&U->max_dist, 4);
    mix(&U->distortion_power, 4);
    const uint64_t pser = d->partition ? d->partition->serial : 0u;
    const uint32_t f[9] = {d->width, d->height, d->max_iters, d->scene_flags, d->math, d->layout, d->shard_index,
                           d->shard_count, d->schedule};
    mix(f, sizeof f);
    mix(&pser, sizeof pser);
    return h | 1u;  // never 0: 0 marks the fresh state's all-zero costs
}

static bool same_launch(const bh_render_desc* a, const bh_render_desc* b) {
    return a->width == b->width && a->height == b->height && a->max_iters == b->max_iters &&
           a->scene_flags == b->scene_flags && a->format == b->format && a->math == b->math &&
           a->layout == b->layout && a->shard_index == b->shard_index && a->shard_count == b->shard_count &&
           a->schedule == b->schedule && a->partition == b->partition;
}

int bh_render(bh_ctx* c, const bh_camera_uniform* cam, const bh_uniforms* U, const bh_render_desc* d,
              void* stream) {
    return bh_render_frames(c, 1u, cam, U, d, stream);
}

// The far-field radius of the root-free step (bh_march.hpp): r^2 beyond which every SDF term of a step
// provably exceeds the root-free test's threshold T = RN(1.125 RN(dtm r) + 0.002) <= 1.1251 dtm R + 0.003
// (R = |p| exact; the roundings of r, dtm r and T are within 2^-21 of R).  For a point at distance R:
//   disc (:121)  >= R / sqrt2 - max(6 rs, 0.02)   (rho^2 + y^2 = R^2: rho or |y| is >= R / sqrt2, and the
//                                                 sdf is >= rho - 6 rs and >= |y| - 0.02)
//   markers      >= R - 10 sqrt2 - 0.5            (the four centres lie at 10 sqrt2 from the origin)
//   photon (:294) >= R - 1.5 rs - 0.075           (its centre lies at 1.5 rs)
// R0 = the largest R at which one of them meets 1.1251 dtm R + 0.003; beyond 1.01 R0 each exceeds the
// threshold by >= 0.01 R0 (0.7071 - 1.1251 dtm) > 0.001 absolute, far above the step's own rounding of
// those terms (relative 2^-21: a few 1e-5 at R ~ 40), so the computed distance exceeds T and the root-free
// test's chain gives dt == dtm r and no surface.  r^2 is compared as computed (within 2^-22 of R^2: inside
// the 1 % margin).  +inf (off) when dtm is too large for the disc bound to ever clear (dtm >= 0.62).
static float sdf_far_r2(float rs, float dtm) {
    const double k = 1.1251 * (double)dtm, a1 = std::sqrt(0.5) - k, a2 = 1.0 - k;
    if (!(a1 > 0.01) || !(rs > 0.0f)) return INFINITY;
    const double R0 = std::max({(std::max(6.0 * rs, 0.02) + 0.003) / a1, (10.0 * std::sqrt(2.0) + 0.5 + 0.003) / a2,
                                (1.5 * rs + 0.075 + 0.003) / a2});
    const double R = 1.01 * R0;
    return std::nextafter((float)(R * R), INFINITY);
}

// A/B switch (diagnostics): BH_NO_SDF_SKIP set => every step evaluates its SDF roots (bh_march.hpp, sdf_skip)
static bool sdf_skip_disabled() {
    static const bool off = std::getenv("BH_NO_SDF_SKIP") != nullptr;
    return off;
}

int bh_render_frames(bh_ctx* c, uint32_t n_frames, const bh_camera_uniform* cams, const bh_uniforms* U,
                     const bh_render_desc* descs, void* stream) {
    if (!c || !cams || !U || !descs || n_frames == 0 || n_frames > BH_MAX_FRAMES) return bad_arg(__func__, __LINE__);
    const bh_render_desc* d = &descs[0];
    const bh_camera_uniform* cam = &cams[0];
    if (!d->out_col) return bad_arg(__func__, __LINE__);
    if (d->width == 0 || d->height == 0 || d->width > 65536u || d->height > 65536u) return bad_arg(__func__, __LINE__);
    if (d->max_iters == 0 || d->max_iters > 65535u) return bad_arg(__func__, __LINE__);
    if (d->format > BH_OUT_BGRA8_SRGB || d->math > BH_MATH_FAST || d->layout > BH_LAYOUT_TILES_RGBM14) return bad_arg(__func__, __LINE__);
    if ((d->schedule & 0xFFu) > BH_SCHED_PERSISTENT || (d->schedule & ~(0xFFu | BH_SCHED_FLAG_STATIC_ORDER | BH_SCHED_FLAG_ISSUE_ORDER | BH_SCHED_FLAG_LATENCY))) return bad_arg(__func__, __LINE__);
    if (d->scene_flags & ~BH_SCENE_DEFAULT) return bad_arg(__func__, __LINE__);
    if (d->shard_count == 0 || d->shard_index >= d->shard_count) return bad_arg(__func__, __LINE__);
    if (d->layout == BH_LAYOUT_ROWMAJOR && d->shard_count != 1) return bad_arg(__func__, __LINE__);
    for (uint32_t i = 0; i < n_frames; ++i) {
        if (!descs[i].out_col || !same_launch(d, &descs[i])) return bad_arg(__func__, __LINE__);
        if (!screen_tri_default(&cams[i])) { g_last_error = "non-default screen triangle"; return BH_ERR_UNSUPPORTED; }
    }
    if ((d->layout == BH_LAYOUT_TILES_RGBM || d->layout == BH_LAYOUT_TILES_RGBM14) &&
        (d->schedule & 0xFFu) == BH_SCHED_PERSISTENT) {
        g_last_error = "BH_LAYOUT_TILES_RGBM(14) needs the tile or pair schedule";
        return BH_ERR_UNSUPPORTED;
    }
    if (d->layout == BH_LAYOUT_TILES_RGBM14 && d->format != BH_OUT_RGBA16F) {
        g_last_error = "BH_LAYOUT_TILES_RGBM14 packs RGBA16F only";
        return BH_ERR_UNSUPPORTED;
    }
    if (n_frames > 1u && (d->schedule & 0xFFu) != BH_SCHED_TILE) {  // one launch per frame
        for (uint32_t i = 0; i < n_frames; ++i) {
            const int st = bh_render_frames(c, 1u, &cams[i], U, &descs[i], stream);
            if (st != BH_OK) return st;
        }
        return BH_OK;
    }

    bh::MarchArgs a;
    std::memset(&a, 0, sizeof(a));
    a.rs = U->rs; a.dtm = U->delta_time_mult; a.max_dist = U->max_dist; a.dp = U->distortion_power;
    a.blackout_eh = U->blackout_eh;
    a.skip_sdf = (U->delta_time_mult > 0.0f && U->rs > 0.0f && U->rs <= 8.0f && !sdf_skip_disabled()) ? 1u : 0u;
    a.far_r2 = a.skip_sdf ? sdf_far_r2(U->rs, U->delta_time_mult) : INFINITY;
    a.width = d->width; a.height = d->height; a.max_iters = d->max_iters; a.scene_flags = d->scene_flags;
    a.format = d->format; a.layout = d->layout;
    a.shard_index = d->shard_index; a.shard_count = d->shard_count;
    a.tiles_x = (d->width + 7u) / 8u; a.tiles_y = (d->height + 7u) / 8u;
    uint64_t nt;
    if (const bh_partition* P = d->partition) {
        if (P->width != d->width || P->height != d->height || P->shard_count != d->shard_count ||
            P->device != c->device || d->layout == BH_LAYOUT_ROWMAJOR) {
            g_last_error = "partition: frame size, shard count, device or layout do not match";
            return BH_ERR_INVALID_ARG;
        }
        if ((d->schedule & 0xFFu) != BH_SCHED_TILE) {
            g_last_error = "a weighted partition needs the tile schedule";
            return BH_ERR_UNSUPPORTED;
        }
        nt = P->count[d->shard_index];
        a.tile_list = P->tile_list + P->offset[d->shard_index];
    } else {
        nt = bh::shard_tile_count(a.tiles_x, a.tiles_y, d->shard_index, d->shard_count);
    }
    if (nt * n_frames > 0xFFFFFFF0ull) return bad_arg(__func__, __LINE__);
    a.n_tiles = (uint32_t)nt;
    // centre-out dispatch blocks of ~one tile row of this shard, centred on the black hole's row
    a.order_block = (uint32_t)((nt + a.tiles_y - 1u) / a.tiles_y);
    a.order_centre = bh_tile_row(cam, d->height);
    a.sky = c->sky; a.srgb_lut = c->lut; a.srgb_enc = c->enc; a.sky_w = c->sky_w; a.sky_h = c->sky_h;
    // k = (DP * RS) * -1.5 (:126); the per-frame fields (camera, c_ps, outputs)
    a.kfac = (a.dp * a.rs) * -1.5f;
    a.rw2 = 1.0f / (2.0f * (float)a.width);
    a.rh2 = 1.0f / (2.0f * (float)a.height);
    a.n_frames = n_frames;
    a.clk = c->clk;
    a.clk_mask = c->clk_mask;
    std::vector<bh::FrameArgs> table;  // n_frames > BH_INLINE_FRAMES: staged in the stream's device table
    if (n_frames > bh::BH_INLINE_FRAMES) table.resize(n_frames);
    bh::FrameArgs* fa = table.empty() ? a.frames : table.data();
    for (uint32_t i = 0; i < n_frames; ++i) frame_args(&cams[i], a.rs, &descs[i], &fa[i]);
    {
        const bh::FrameArgs& F = fa[0];
        for (int k = 0; k < 3; ++k) {
            a.pos[k] = F.pos[k]; a.c0[k] = F.c0[k]; a.c1[k] = F.c1[k]; a.c2[k] = F.c2[k]; a.cps[k] = F.cps[k];
        }
        a.out_col = F.out_col; a.out_blackout = F.out_blackout;
        a.dbg_n_rk = F.dbg_n_rk; a.dbg_fate = F.dbg_fate; a.dbg_steps = F.dbg_steps;
    }
    if (a.n_tiles == 0) return BH_OK;

    DeviceScope dev(c->device);
    if (dev.err != hipSuccess) return hip_fail(dev.err, "hipSetDevice");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uint32_t sched = d->schedule & 0xFFu;
    if (!table.empty()) {
        const int st = stage_frame_table(c, s, table.data(), n_frames, &a.frame_table);
        if (st != BH_OK) return st;
    }
    bh_ctx::OrderState* os = nullptr;
    if (sched == BH_SCHED_TILE && !(d->schedule & BH_SCHED_FLAG_STATIC_ORDER)) {
        // temporal order of this (geometry, shard, stream): allocated at its first render only
        int st = order_state(c, d, nt, s, stream_capturing(s), &os);
        if (st != BH_OK) return st;
        if (!os->valid) {
            // all costs 0 (one bucket, the uncounted last) and an empty histogram: consistent
            hipError_t he = hipMemsetAsync(os->counters, 0, bh::ORDER_WORDS * sizeof(uint32_t), s);
            if (he == hipSuccess) he = hipMemsetAsync(os->tile_cost, 0, nt, s);
            if (he != hipSuccess) return hip_fail(he, "temporal order reset");
            os->valid = true;
            os->cost_key = 0u;
            os->order_key = ~0ull;
        }
        // The order build consumes the histogram the last march accumulated (and zeroes the counters), and
        // the march accumulates the next: at every launch boundary the counters hold the histogram of the
        // costs in tile_cost, also across graph replays, which repeat a captured launch as it was.  A launch
        // whose frame repeats the one the order was learned from (its key equals both the order's and the
        // costs') skips the pair: no build, and a march that writes no costs -- the pending histogram still
        // describes the unchanged costs.  The host's keys only decide the skip; a replay that changed the
        // buffers behind them costs at most a stale order, never a disagreement.  BH_ORDER_ALWAYS (A/B):
        // build and write on every launch, as before round 5.
        static const bool always = std::getenv("BH_ORDER_ALWAYS") != nullptr;
        const uint64_t key = frame_cost_key(&cams[0], U, d);
        const bool repeat = !always && os->order_key == os->cost_key && os->cost_key == key;
        if (!repeat) {
            int oe = bh_launch_build_order(os->tile_cost, a.n_tiles, a.order_block, a.order_centre, os->counters,
                                           os->order, s);
            if (oe != 0) { os->valid = false; return hip_fail((hipError_t)oe, "order kernels"); }
            os->order_key = os->cost_key;
            os->cost_key = key;
        }
        a.order = os->order;
        a.tile_cost = repeat ? nullptr : os->tile_cost;
        a.order_tot = repeat ? nullptr : os->counters;
    }
    int e = d->math != BH_MATH_EXACT ? bh_launch_march_fast(a, sched, c->counters, c->grid_fast, s)
            : march_variant_issue_order(d, a.n_tiles, a.n_frames, c->cus)
                ? bh_launch_march_exact(a, sched, c->counters, c->grid_exact, s)
                : bh_launch_march_exact_lat(a, sched, c->counters, c->grid_exact, s);
    if (e != 0) {
        // the costs and their histogram are written together by the march kernel; without it they
        // may disagree, so the next frame of this state starts the temporal order afresh
        if (os) os->valid = false;
        return hip_fail((hipError_t)e, "march kernel launch");
    }
    return BH_OK;
}

int bh_set_clock_probe(bh_ctx* c, uint64_t* acc, uint32_t stride) {
    if (!c || (acc && (stride == 0u || (stride & (stride - 1u)) != 0u))) return bad_arg(__func__, __LINE__);
    c->clk = reinterpret_cast<unsigned long long*>(acc);
    c->clk_mask = acc ? stride - 1u : 0u;
    return BH_OK;
}

int bh_tiles_unpack(const void* packed, void* out, uint32_t width, uint32_t height, uint32_t shard_count,
                    uint64_t shard_stride_tiles, uint32_t bpp, void* stream) {
    if (!packed || !out || width == 0 || height == 0 || shard_count == 0) return bad_arg(__func__, __LINE__);
    if (bpp != 4 && bpp != 8 && bpp != 16) return bad_arg(__func__, __LINE__);
    for (uint32_t k = 0; k < shard_count; ++k)
        if (bh::shard_tile_count((width + 7u) / 8u, (height + 7u) / 8u, k, shard_count) > shard_stride_tiles)
            return bad_arg(__func__, __LINE__);
    int e = bh_launch_tiles_unpack(packed, out, width, height, shard_count, shard_stride_tiles, bpp,
                                   reinterpret_cast<hipStream_t>(stream));
    if (e != 0) return hip_fail((hipError_t)e, "tiles unpack launch");
    return BH_OK;
}

// an RGBM unpack's format: a bh_out_format, or BH_OUT_RGBA16F | BH_UNPACK_RGBM14
static bool unpack_format_ok(uint32_t format) {
    return format <= BH_OUT_BGRA8_SRGB || format == (BH_OUT_RGBA16F | BH_UNPACK_RGBM14);
}

int bh_tiles_unpack_rgb_rows(const void* packed, void* out, uint32_t width, uint32_t height, uint32_t shard_count,
                             uint64_t shard_stride_tiles, uint32_t format, uint32_t rows_in_flight, void* stream) {
    if (!packed || !out || width == 0 || height == 0 || shard_count == 0) return bad_arg(__func__, __LINE__);
    if (format > BH_OUT_BGRA8_SRGB) return bad_arg(__func__, __LINE__);
    for (uint32_t k = 0; k < shard_count; ++k)
        if (bh::shard_tile_count((width + 7u) / 8u, (height + 7u) / 8u, k, shard_count) > shard_stride_tiles)
            return bad_arg(__func__, __LINE__);
    int e = bh_launch_tiles_unpack_rgb(packed, out, width, height, shard_count, shard_stride_tiles, format,
                                       rows_in_flight, reinterpret_cast<hipStream_t>(stream));
    if (e != 0) return hip_fail((hipError_t)e, "tiles unpack launch");
    return BH_OK;
}

int bh_tiles_unpack_rgb(const void* packed, void* out, uint32_t width, uint32_t height, uint32_t shard_count,
                        uint64_t shard_stride_tiles, uint32_t format, void* stream) {
    return bh_tiles_unpack_rgb_rows(packed, out, width, height, shard_count, shard_stride_tiles, format, 0u, stream);
}

int bh_tiles_unpack_rgbm(const void* packed, void* out, void* out_bo, uint32_t width, uint32_t height,
                         uint32_t shard_count, uint64_t shard_stride_tiles, uint32_t format, uint32_t rows_in_flight,
                         void* stream) {
    if (!packed || !out || width == 0 || height == 0 || shard_count == 0) return bad_arg(__func__, __LINE__);
    if (!unpack_format_ok(format)) return bad_arg(__func__, __LINE__);
    for (uint32_t k = 0; k < shard_count; ++k)
        if (bh::shard_tile_count((width + 7u) / 8u, (height + 7u) / 8u, k, shard_count) > shard_stride_tiles)
            return bad_arg(__func__, __LINE__);
    int e = bh_launch_tiles_unpack_rgbm(packed, out, out_bo, width, height, shard_count, shard_stride_tiles, nullptr,
                                        format, rows_in_flight, reinterpret_cast<hipStream_t>(stream));
    if (e != 0) return hip_fail((hipError_t)e, "tiles unpack launch");
    return BH_OK;
}

namespace {
// Owner of each residue (tx + 3 ty) mod M, M = sum(weights): smooth weighted round robin, so each shard's
// residues are spread evenly over the M.  Empty if the weights are unusable.
std::vector<uint32_t> partition_owners(uint32_t S, const uint32_t* w) {
    uint64_t M = 0;
    for (uint32_t k = 0; k < S; ++k) M += w[k];
    if (M == 0 || M > 4096) return {};
    std::vector<uint32_t> owner(M);
    std::vector<int64_t> cw(S, 0);
    for (uint64_t v = 0; v < M; ++v) {
        uint32_t best = 0;
        for (uint32_t k = 0; k < S; ++k) {
            cw[k] += w[k];
            if (cw[k] > cw[best]) best = k;
        }
        owner[v] = best;
        cw[best] -= (int64_t)M;
    }
    return owner;
}
}  // namespace

int bh_partition_map(uint32_t width, uint32_t height, uint32_t S, const uint32_t* weights, uint32_t* owner_out,
                     uint32_t* index_out) {
    if (width == 0 || height == 0 || width > 65536u || height > 65536u || S == 0 || S > 256 || !weights)
        return bad_arg(__func__, __LINE__);
    const std::vector<uint32_t> owner = partition_owners(S, weights);
    if (owner.empty()) return bad_arg(__func__, __LINE__);
    const uint32_t M = (uint32_t)owner.size(), tx_n = (width + 7u) / 8u, ty_n = (height + 7u) / 8u;
    std::vector<uint32_t> next(S, 0);
    for (uint32_t ty = 0; ty < ty_n; ++ty)
        for (uint32_t tx = 0; tx < tx_n; ++tx) {
            const uint32_t k = owner[(tx + 3ull * ty) % M];
            const size_t t = (size_t)ty * tx_n + tx;
            if (owner_out) owner_out[t] = k;
            if (index_out) index_out[t] = next[k];
            ++next[k];
        }
    return BH_OK;
}

int bh_partition_create(uint32_t width, uint32_t height, uint32_t S, const uint32_t* weights, int device,
                        bh_partition** out) {
    if (!out) return bad_arg(__func__, __LINE__);
    *out = nullptr;
    const uint32_t tx_n = (width + 7u) / 8u, ty_n = (height + 7u) / 8u;
    const size_t n = (size_t)tx_n * ty_n;
    if (n >= (1u << 24)) return bad_arg(__func__, __LINE__);  // packed indices carry 24 bits
    std::vector<uint32_t> owner(n), index(n);
    int st = bh_partition_map(width, height, S, weights, owner.data(), index.data());
    if (st != BH_OK) return st;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return BH_ERR_NO_DEVICE;
    bh_partition* P = new (std::nothrow) bh_partition;
    if (!P) return BH_ERR_OUT_OF_MEMORY;
    P->width = width; P->height = height; P->shard_count = S; P->tiles_x = tx_n; P->tiles_y = ty_n;
    P->device = device;
    P->serial = ++g_partition_serial;
    P->count.assign(S, 0);
    for (size_t t = 0; t < n; ++t) ++P->count[owner[t]];
    P->offset.assign(S, 0);
    for (uint32_t k = 1; k < S; ++k) P->offset[k] = P->offset[k - 1] + P->count[k - 1];
    std::vector<uint32_t> list(n), loc(n);
    for (size_t t = 0; t < n; ++t) {
        const uint32_t k = owner[t];
        list[P->offset[k] + index[t]] = (uint32_t)(t % tx_n) | (uint32_t)(t / tx_n) << 16;
        loc[t] = index[t] | k << 24;
    }
    DeviceScope dev(device);
    hipError_t e = dev.err;
    if (e != hipSuccess || (e = hipMalloc(&P->tile_list, n * 4)) != hipSuccess || (e = hipMalloc(&P->tile_loc, n * 4)) != hipSuccess ||
        (e = hipMemcpy(P->tile_list, list.data(), n * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(P->tile_loc, loc.data(), n * 4, hipMemcpyHostToDevice)) != hipSuccess) {
        st = e == hipErrorOutOfMemory ? BH_ERR_OUT_OF_MEMORY : hip_fail(e, "partition tables");
        if (P->tile_list) (void)hipFree(P->tile_list);
        if (P->tile_loc) (void)hipFree(P->tile_loc);
        delete P;
        return st;
    }
    *out = P;
    return BH_OK;
}

int bh_partition_destroy(bh_partition* P) {
    if (!P) return BH_OK;
    {
        DeviceScope dev(P->device);
        if (P->tile_list) (void)hipFree(P->tile_list);
        if (P->tile_loc) (void)hipFree(P->tile_loc);
    }
    delete P;
    return BH_OK;
}

int64_t bh_partition_tile_count(const bh_partition* P, uint32_t shard_index) {
    if (!P || shard_index >= P->shard_count) return bad_arg(__func__, __LINE__);
    return P->count[shard_index];
}

int bh_tiles_unpack_rgbm_partition(const void* packed, void* out, void* out_bo, const bh_partition* P,
                                   uint64_t shard_stride_tiles, uint32_t format, uint32_t rows_in_flight,
                                   void* stream) {
    if (!packed || !out || !P || !unpack_format_ok(format)) return bad_arg(__func__, __LINE__);
    for (uint32_t k = 0; k < P->shard_count; ++k)
        if (P->count[k] > shard_stride_tiles) return bad_arg(__func__, __LINE__);
    int e = bh_launch_tiles_unpack_rgbm(packed, out, out_bo, P->width, P->height, P->shard_count, shard_stride_tiles,
                                        P->tile_loc, format, rows_in_flight, reinterpret_cast<hipStream_t>(stream));
    if (e != 0) return hip_fail((hipError_t)e, "tiles unpack launch");
    return BH_OK;
}

int64_t bh_tile_bytes(uint32_t layout, uint32_t format) {
    if (format > BH_OUT_BGRA8_SRGB) return bad_arg(__func__, __LINE__);
    const int64_t bpp = format == BH_OUT_RGBA32F ? 16 : format == BH_OUT_RGBA16F ? 8 : 4;
    switch (layout) {
        case BH_LAYOUT_TILES: return 64 * bpp;
        case BH_LAYOUT_TILES_RGB: return 48 * bpp;
        case BH_LAYOUT_TILES_RGBM: return 48 * bpp + 8;
        case BH_LAYOUT_TILES_RGBM14: return format == BH_OUT_RGBA16F ? 344 : BH_ERR_UNSUPPORTED;
        default: return bad_arg(__func__, __LINE__);
    }
}

}  // extern "C"
