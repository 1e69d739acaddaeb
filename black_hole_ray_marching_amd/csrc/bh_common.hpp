// bh_common.hpp — host/device shared definitions for the geodesic ray-marcher (no math here).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/bh_render.h"

namespace bh {

// Frames whose arguments travel inline in the kernel argument; a bh_render_frames call of more
// (up to BH_MAX_FRAMES) stages them in a device table (bh_host.cpp, FrameTable).
constexpr uint32_t BH_INLINE_FRAMES = 32;
static_assert(BH_INLINE_FRAMES <= BH_MAX_FRAMES, "inline frames");

// The per-frame part of a launch that renders several frames (bh_render_frames): camera, the
// photon-sphere centre derived from its position, and the frame's outputs.
struct FrameArgs {
    float pos[3];
    float c0[3], c1[3], c2[3];
    float cps[3];
    void* out_col;
    void* out_blackout;
    uint16_t* dbg_n_rk;
    uint8_t* dbg_fate;
    uint16_t* dbg_steps;
};

// Everything one launch needs, passed by value as the kernel argument (lives in SGPRs / kernarg).
// The per-frame fields (pos, c0..c2, cps, outputs) are frame 0's; a multi-frame launch (n_frames > 1,
// tile schedule) also carries every frame's in `frames` and each wave selects its own.
struct MarchArgs {
    // camera uniform (src/black_hole_maybe.wgsl:9-17): ro0 and the three interpolated corner rays
    float pos[3];
    float c0[3], c1[3], c2[3];
    // Uniforms (src/black_hole_maybe.wgsl:58-69)
    float rs, dtm, max_dist, dp;
    uint32_t blackout_eh;
    uint32_t skip_sdf;         // the root-free step may run (bh_march.hpp, sdf_skip: dtm > 0, 0 < rs <= 8)
    float far_r2;              // r^2 beyond which a step needs no SDF argument (bh_host.cpp sdf_far_r2; +inf: off)
    // unused: the per-term radii of a root-free-step variant measured slower and removed;
    // kept so that the kernel argument layout -- and the kernels' machine code -- stay those measured
    float reserved_[3];
    // frame
    uint32_t width, height, max_iters, scene_flags;
    uint32_t format, layout;
    uint32_t shard_index, shard_count;
    uint32_t tiles_x, tiles_y;
    uint32_t n_tiles;          // tiles owned by this shard (= grid work items)
    uint32_t order_block;      // centre-out dispatch: shard-local tiles permuted in blocks of this
    uint32_t order_centre;     //   many tiles (~ one tile row), starting at block order_centre
    const uint32_t* order;     // optional dispatch order (slot -> shard-local tile), else centre-out
    const uint32_t* tile_list; // optional (weighted partition): shard-local tile -> tx | ty << 16
    uint8_t* tile_cost;        // optional output: per shard-local tile, min(255, max n_rk / 2)
    uint32_t* order_tot;       // with tile_cost: per-bucket tile counts of those costs (buckets < B-1)
    // per-frame invariants, computed on the host with the same correctly rounded f32 ops as the
    // oracle: photon-sphere centre -normalize(ro0) * 1.5 * RS (:294) and (DP * RS) * -1.5 (:126)
    float cps[3];
    float kfac;
    // RN(1 / (2W)) and RN(1 / (2H)): the reciprocals of vs_main's interpolation denominators (IEEE on the
    // host; equal to crm::rcp_refined of 2W, 2H, which is RN(1/d) for every normal d)
    float rw2, rh2;
    // sky (Rgba8UnormSrgb texels as packed u32, little endian: r | g<<8 | b<<16 | a<<24)
    const uint32_t* sky;
    const float* srgb_lut;     // 256 entries, sRGB byte -> linear
    const float* srgb_enc;     // 257 thresholds of the BGRA8 sRGB encode (bh_srgb.hpp)
    uint32_t sky_w, sky_h;
    // outputs
    void* out_col;
    void* out_blackout;
    uint16_t* dbg_n_rk;
    uint8_t* dbg_fate;
    uint16_t* dbg_steps;
    // frames of one launch (bh_render_frames): wave slot s marches frame s % n_frames, tile s / n_frames;
    // up to BH_INLINE_FRAMES of them inline, more from a device table (frame_table, else null)
    uint32_t n_frames;
    const FrameArgs* frame_table;
    // shader-clock probe (bh_set_clock_probe): per-XCD accumulators, sampled slots: (slot + slot / 256) & clk_mask == 0
    unsigned long long* clk;
    uint32_t clk_mask;
    FrameArgs frames[BH_INLINE_FRAMES];
};
// passed by value: the kernel argument segment holds at most 4 KiB (with the persistent kernel's
// extra pointer)
static_assert(sizeof(MarchArgs) + 8 <= 4096, "MarchArgs must fit the kernel argument segment");

// Shard ownership: tile (tx, ty) belongs to shard (tx + 3*ty) % S (SURVEY §8e diagonal interleave).
// Row ty's first owned column for shard k.
__host__ __device__ inline uint32_t shard_row_start(uint32_t ty, uint32_t k, uint32_t S) {
    // (k - 3*ty) mod S, computed without negatives
    uint32_t m = (3u * (ty % S)) % S;
    return (k + S - m) % S;
}
__host__ __device__ inline uint32_t shard_row_count(uint32_t tiles_x, uint32_t ty, uint32_t k, uint32_t S) {
    uint32_t st = shard_row_start(ty, k, S);
    return st < tiles_x ? (tiles_x - st + S - 1u) / S : 0u;
}
// Tiles owned in one full period of rows.  Period P = S / gcd(S, 3).
__host__ __device__ inline uint32_t shard_period(uint32_t S) { return (S % 3u == 0u) ? S / 3u : S; }

__host__ __device__ inline uint64_t shard_tile_count(uint32_t tiles_x, uint32_t tiles_y, uint32_t k, uint32_t S) {
    const uint32_t P = shard_period(S);
    uint64_t per = 0;
    for (uint32_t r = 0; r < P && r < tiles_y; ++r) per += shard_row_count(tiles_x, r, k, S);
    uint64_t full = tiles_y / P, n = full * per;
    for (uint32_t r = 0; r < tiles_y % P; ++r) n += shard_row_count(tiles_x, r, k, S);
    return n;
}

// The rows of one period of shard k, walked without divisions (these run once per wave in the
// march kernel and once per tile in the unpack; the division-per-row form cost ~1000 VALU
// instructions per tile at S = 8).  Row r of a period starts at column st = (k - 3r) mod S and
// owns q0 + (st < r0) tiles, with tiles_x = q0*S + r0.
struct ShardRows {
    uint32_t k, S, q0, r0, m;  // m = 3r mod S of the current row
    __host__ __device__ ShardRows(uint32_t tiles_x, uint32_t k_, uint32_t S_) : k(k_), S(S_), m(0u) {
        q0 = tiles_x / S; r0 = tiles_x - q0 * S;
    }
    __host__ __device__ uint32_t start() const { return k >= m ? k - m : k + S - m; }
    __host__ __device__ uint32_t count() const { return q0 + (start() < r0 ? 1u : 0u); }
    __host__ __device__ void next() { m += 3u; while (m >= S) m -= S; }
};

// Shard-local tile index t -> global tile coordinates.
__host__ __device__ inline void shard_tile_coords(uint32_t t, uint32_t tiles_x, uint32_t k, uint32_t S,
                                                  uint32_t* tx, uint32_t* ty) {
    if (S == 1u) { *ty = t / tiles_x; *tx = t - *ty * tiles_x; return; }
    const uint32_t P = shard_period(S);
    uint32_t per = 0;
    ShardRows R(tiles_x, k, S);
    for (uint32_t r = 0; r < P; ++r, R.next()) per += R.count();
    const uint32_t period = t / per;
    uint32_t rem = t - period * per, row = 0;
    ShardRows Q(tiles_x, k, S);
    for (; row + 1u < P; ++row, Q.next()) {
        const uint32_t c = Q.count();
        if (rem < c) break;
        rem -= c;
    }
    *ty = period * P + row;
    *tx = Q.start() + rem * S;
}

// Inverse of shard_tile_coords: global tile (tx, ty) -> its shard and its shard-local index.
__host__ __device__ inline uint32_t shard_tile_index(uint32_t tx, uint32_t ty, uint32_t tiles_x, uint32_t S,
                                                     uint32_t* shard) {
    const uint32_t k = (tx + 3u * (ty % S)) % S;
    *shard = k;
    if (S == 1u) return ty * tiles_x + tx;
    const uint32_t P = shard_period(S);
    const uint32_t rp = ty % P;
    uint32_t per = 0, pre = 0;
    ShardRows R(tiles_x, k, S);
    for (uint32_t r = 0; r < P; ++r, R.next()) {
        const uint32_t c = R.count();
        per += c;
        pre += r < rp ? c : 0u;
    }
    return (ty / P) * per + pre + tx / S;  // tx = row start + j*S with the row start < S
}

// Centre-out dispatch order (a bijection of [0, n)): the shard-local tile range is cut into blocks
// of L tiles (~ one tile row); block slot k of the dispatch takes block c, c+1, c-1, c+2, c-2, ...
// (clipped to the range) and the partial tail block stays last.  c is the block holding the black
// hole's projected screen row, so the photon-ring tiles -- where the capped "Zeno" rays that run
// the full 512-step chain live -- start first and their serial chains overlap the rest of the frame.
// Only the order changes, never a result.
__host__ __device__ inline uint32_t centre_out(uint32_t b, uint32_t n, uint32_t L, uint32_t c) {
    if (L == 0u) return b;
    const uint32_t nb = n / L;
    const uint32_t j = b / L, i = b - j * L;
    if (j >= nb) return b;
    if (c >= nb) c = nb - 1u;
    const uint32_t m = c < nb - 1u - c ? c : nb - 1u - c;  // full pairs on both sides
    uint32_t J;
    if (j == 0u) J = c;
    else if (j <= 2u * m) J = (j & 1u) ? c + (j + 1u) / 2u : c - j / 2u;
    else J = (c - m == 0u) ? c + m + (j - 2u * m) : c - m - (j - 2u * m);
    return J * L + i;
}

}  // namespace bh

namespace bh {
// Dispatch-order buckets by the previous frame's per-tile cost (max n_rk / 2): expensive first.
constexpr uint32_t ORDER_BUCKETS = 6;
// Words of a temporal-order state's counters: [0, B-1) the cost histogram, [B, 2B) the order kernel's
// cursors, [2B] its block ticket.
constexpr uint32_t ORDER_WORDS = 2 * ORDER_BUCKETS + 1;
__host__ __device__ inline uint32_t cost_bucket(uint32_t c) {
    return c >= 128u ? 0u : c >= 64u ? 1u : c >= 32u ? 2u : c >= 20u ? 3u : c >= 12u ? 4u : 5u;
}

// Max over the wave's 64 lanes, every lane active: an inclusive DPP scan (row_shr 1/2/4/8 within each
// 16-lane row, then row_bcast:15 and row_bcast:31 across rows) leaves the max in lane 63.  Out-of-range
// DPP sources read 0, the identity of an unsigned max.  (__shfl_xor: six ds_bpermute round trips and
// ~36 VALU of index arithmetic.)
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_max_step(uint32_t v) {
    return max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, false));
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = dpp_max_step<0x111>(v);         // row_shr:1
    v = dpp_max_step<0x112>(v);         // row_shr:2
    v = dpp_max_step<0x114>(v);         // row_shr:4
    v = dpp_max_step<0x118>(v);         // row_shr:8
    v = dpp_max_step<0x142, 0xa>(v);    // row_bcast:15 into rows 1 and 3
    v = dpp_max_step<0x143, 0xc>(v);    // row_bcast:31 into rows 2 and 3
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
}  // namespace bh

// Launchers (defined in the .hip translation units).
extern "C" __attribute__((visibility("hidden"))) int bh_launch_march_exact(const bh::MarchArgs& a, uint32_t schedule,
                                                                         uint32_t* counters, uint32_t grid,
                                                                         hipStream_t s);
extern "C" __attribute__((visibility("hidden"))) int bh_launch_march_exact_lat(const bh::MarchArgs& a, uint32_t schedule,
                                                                             uint32_t* counters, uint32_t grid,
                                                                             hipStream_t s);
extern "C" __attribute__((visibility("hidden"))) int bh_launch_march_fast(const bh::MarchArgs& a, uint32_t schedule,
                                                                        uint32_t* counters, uint32_t grid,
                                                                        hipStream_t s);
extern "C" __attribute__((visibility("hidden"))) int bh_march_blocks_per_cu_exact(void);
extern "C" __attribute__((visibility("hidden"))) int bh_march_blocks_per_cu_fast(void);
extern "C" __attribute__((visibility("hidden"))) int bh_launch_build_order(const uint8_t* cost, uint32_t n_tiles,
                                                                         uint32_t block, uint32_t centre,
                                                                         uint32_t* counters, uint32_t* order,
                                                                         hipStream_t s);
extern "C" __attribute__((visibility("hidden"))) int bh_launch_tiles_unpack_rgbm(const void* packed, void* out, void* out_bo,
                                                                               uint32_t width, uint32_t height,
                                                                               uint32_t shard_count, uint64_t stride_tiles,
                                                                               const uint32_t* tile_loc,
                                                                               uint32_t format, uint32_t rows_in_flight,
                                                                               hipStream_t s);
extern "C" __attribute__((visibility("hidden"))) int bh_launch_tiles_unpack_rgb(const void* packed, void* out, uint32_t width,
                                                                              uint32_t height, uint32_t shard_count,
                                                                              uint64_t stride_tiles, uint32_t format, uint32_t rows_in_flight,
                                                                              hipStream_t s);
// base codes of the table form of the sRGB encoder (bh_srgb.hpp), built from its 257 thresholds
extern "C" __attribute__((visibility("hidden"))) void bh_srgb_bucket_table(const float* T257, uint8_t* B);
extern "C" __attribute__((visibility("hidden"))) bool bh_srgb_code_table(const float* T257, uint32_t* E);
// bh_bloom.hip pass shaders (bh::bloom::Shader)
constexpr uint32_t bh_bloom_shader_copy = 0, bh_bloom_shader_down = 1, bh_bloom_shader_up = 2, bh_bloom_shader_remix = 3;
// the separable plan of an 8-tap pass (bh_bloom.hip): 8 * (ow + oh) entries of 4 words; returns the largest
// block footprint side (or -1)
extern "C" __attribute__((visibility("hidden"))) int bh_bloom_sep_plan(uint32_t ow, uint32_t oh, uint32_t tw,
                                                                     uint32_t th, uint32_t rx, uint32_t ry,
                                                                     uint32_t* outp, uint32_t org);
// an up pass from its separable plan with an epilogue (bh_bloom.hip SepEpi: 0 plain, 1 Y, 2 final)
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_sep(const float* lut, const float* enc,
                                                                        const uint8_t* buckets, const uint32_t* codes,
                                                                        const uint32_t* a, uint32_t aw, uint32_t ah,
                                                                        uint32_t rx, uint32_t ry,
                                                                        const uint32_t* sep, int ext, uint32_t epi,
                                                                        const uint32_t* own0, const uint32_t* own1,
                                                                        const uint32_t* same, uint32_t* out, uint32_t* aux,
                                                                        uint32_t ow, uint32_t oh, uint32_t org, bool fix,
                                                                        const uint32_t* stc, uint32_t* strips,
                                                                        uint32_t strip_w, bool* strips_written,
                                                                        hipStream_t s);
// the fix-up pass of a fused epilogue; stc / strips: the final epilogue's column strips (the up pass wrote them)
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_fixup(const float* lut, const float* enc,
                                                                          const uint8_t* buckets, const uint32_t* codes,
                                                                          uint32_t epi, const uint32_t* a, const uint32_t* b,
                                                                          const uint32_t* c, const uint32_t* same,
                                                                          const uint32_t* list, uint32_t n_cols,
                                                                          uint32_t n_rows, uint32_t* out, uint32_t w,
                                                                          uint32_t h, int32_t residual_org, const uint32_t* recs,
                                                                          const uint32_t* stc, const uint32_t* strips,
                                                                          uint32_t strip_w, hipStream_t s);
// the column strips' table of a same-size plan's inexact columns; returns the number of strip columns
extern "C" __attribute__((visibility("hidden"))) uint32_t bh_bloom_strip_table(uint32_t w, const uint32_t* list, uint32_t nc,
                                                                         uint32_t* stc);
// the fix-up kernel's records of a list (8 words per entry: the index and the plan entries of it and its neighbours)
extern "C" __attribute__((visibility("hidden"))) void bh_bloom_fixup_records(uint32_t w, uint32_t h, const uint32_t* plan,
                                                                           const uint32_t* list, uint32_t nc, uint32_t nr,
                                                                           uint32_t* out);
// two downsamples a -> mw x mh -> out in one pass (the intermediate level not stored)
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_down2(const float* lut, const float* enc,
                                                                          const uint8_t* buckets, const uint32_t* codes,
                                                                          const uint32_t* a, uint32_t aw, uint32_t ah,
                                                                          uint32_t mw, uint32_t mh, uint32_t* out,
                                                                          uint32_t ow, uint32_t oh, hipStream_t s);
// the same-size plan of a w x h frame (bh_bloom.hip): (w + h) uint2 entries; the plan remixes
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_same_plan(uint32_t w, uint32_t h, uint32_t* outp);
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_remix_plan(const float* lut, const float* enc,
                                                                               const uint8_t* buckets,
                                                                               const uint32_t* codes, const uint32_t* a,
                                                                               const uint32_t* b, const uint32_t* plan,
                                                                               uint32_t* out, uint32_t w, uint32_t h,
                                                                               hipStream_t s);
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_same_copy(const float* lut, const float* enc,
                                                                              const uint8_t* buckets,
                                                                              const uint32_t* codes, const uint32_t* src,
                                                                              const uint32_t* plan, uint32_t* out,
                                                                              uint32_t w, uint32_t h, hipStream_t s);
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_remix2_plan(const float* lut, const float* enc,
                                                                                const uint8_t* buckets,
                                                                                const uint32_t* codes,
                                                                                const uint32_t* col, const uint32_t* Y,
                                                                                const uint32_t* Bt, const uint32_t* plan,
                                                                                uint32_t* out, uint32_t w, uint32_t h,
                                                                                hipStream_t s);
// host-side bound checks of the bloom kernels' index arithmetic (bh_bloom.hip): a separable plan for the form
// bh_launch_bloom_sep takes, a same-size plan with its fix-up list; false with the first violation in *why.
// Dry mode (bh_bloom_check): between begin and end the bloom launchers check their launch instead of launching.
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_sep_verify(uint32_t ow, uint32_t oh, uint32_t tw,
                                                                        uint32_t th, uint32_t rx, uint32_t ry,
                                                                        const uint32_t* plan, int ext, uint32_t org, bool fix,
                                                                        std::string* why);
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_sep_fix_ok(int ext, uint32_t ow, uint32_t oh, uint32_t epi);
// the quad grid origin of the in-block fix for a same-size plan, and its residual (crossing) columns / rows
extern "C" __attribute__((visibility("hidden"))) uint32_t bh_bloom_same_org(uint32_t w, uint32_t h, const uint32_t* plan,
                                                                          std::vector<uint32_t>* cols,
                                                                          std::vector<uint32_t>* rows,
                                                                          std::vector<uint32_t>* cols2,
                                                                          std::vector<uint32_t>* rows2);
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_same_verify(uint32_t w, uint32_t h, const uint32_t* plan,
                                                                         uint32_t nc, uint32_t nr, std::string* why);
// bh_host.cpp for the other host translation units: the thread's last error, an argument failure, a ctx's device
extern "C" __attribute__((visibility("hidden"))) void bh_set_last_error(const std::string& msg);
extern "C" __attribute__((visibility("hidden"))) int bh_bad_arg(const char* fn, int line);
extern "C" __attribute__((visibility("hidden"))) int bh_ctx_device(const bh_ctx* c);
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_records_verify(uint32_t w, uint32_t h, const uint32_t* plan,
                                                                            const uint32_t* list, uint32_t nc, uint32_t nr,
                                                                            const uint32_t* rec, const uint32_t* stc,
                                                                            uint32_t strip_w, std::string* why);
extern "C" __attribute__((visibility("hidden"))) void bh_bloom_dry_begin(void);
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_dry_end(uint64_t* launches, uint64_t* checks,
                                                                     std::string* fail, std::string* plan);
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_dry(void);
// whether bh_launch_bloom_pass runs an up pass of this shape from its separable plan (bh_bloom.hip)
extern "C" __attribute__((visibility("hidden"))) bool bh_bloom_up_uses_sep(uint32_t ow, uint32_t oh, uint32_t aw,
                                                                         uint32_t ah, uint32_t rx, uint32_t ry);
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_pass(uint32_t shader, const float* lut,
                                                                         const float* enc, const uint8_t* buckets,
                                                                         const uint32_t* codes, const uint32_t* a,
                                                                         uint32_t aw, uint32_t ah, const uint32_t* b,
                                                                         uint32_t rx, uint32_t ry, uint32_t* out,
                                                                         uint32_t ow, uint32_t oh, const uint32_t* sep, int sep_ext,
                                                                         hipStream_t s);
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_y(const float* lut, const float* enc,
                                                                      const uint8_t* buckets, const uint32_t* codes,
                                                                      const uint32_t* X, uint32_t* Y, uint32_t w,
                                                                      uint32_t h, uint32_t* d2out, bool* d2_done,
                                                                      hipStream_t s);
extern "C" __attribute__((visibility("hidden"))) int bh_launch_bloom_final(const float* lut, const float* enc,
                                                                          const uint8_t* buckets, const uint32_t* codes,
                                                                          const uint32_t* col, const uint32_t* Y,
                                                                          const uint32_t* U0, uint32_t rx, uint32_t ry,
                                                                          uint32_t* out, uint32_t w, uint32_t h,
                                                                          hipStream_t s);
extern "C" __attribute__((visibility("hidden"))) int bh_launch_tiles_unpack(const void* packed, void* out, uint32_t width, uint32_t height,
                                      uint32_t shard_count, uint64_t shard_stride_tiles,
                                      uint32_t bytes_per_pixel, hipStream_t s);
