// bh_tiles.hip — scatter gathered tile-packed shards back into a row-major frame (rank 0 after the
// RCCL gather), and the temporal dispatch order of the tile schedule.  The unpack is
// pure byte movement (HBM-bound): whole packed tiles in, full frame-row segments out.
#include "bh_common.hpp"

namespace bh {

// Unpack is organised by OUTPUT: a workgroup covers UNPACK_SPAN horizontally adjacent tiles of one
// tile row (256 x 8 pixels).  A shard's tiles of one row are consecutive in its packed buffer, so
// the workgroup reads each shard's share of the span as one contiguous run (UNPACK_SPAN / S tiles)
// into LDS, then writes 8 full 256-pixel frame row segments (one 512-B store per wave instruction
// for RGBA16F).  Measured at the N=8 frame (11584x5792 RGBA16F, 0.94 GB moved): walking the packed
// buffer instead (consecutive waves = consecutive tiles of one shard, 8 rows x 64 B per store) ran
// at 635 GB/s; output-major with 4 tiles per workgroup at 1.6-1.9 TB/s, limited by reading 8
// shards' runs of 1 tile each; a plain copy of the same bytes runs at 5.2 TB/s.
constexpr uint32_t UNPACK_SPAN = 32;
struct UnpackGrid {
    uint32_t width, height, tiles_x, shard_count;
    uint64_t stride_tiles;
    const uint32_t* tile_loc;  // weighted partition: tile -> its packed index | shard << 24 (else the interleave)
};
template <uint32_t BPP> struct PixelT;
template <> struct PixelT<16> { using T = uint4; };
template <> struct PixelT<8> { using T = uint2; };
template <> struct PixelT<4> { using T = uint32_t; };

// PLANAR: BH_LAYOUT_TILES_RGB of the format whose pixel is BPP bytes (three planes of 64 channel
// values of BPP/4 bytes, alpha restored); else BH_LAYOUT_TILES (whole pixels, any format).
// MASK (with PLANAR): BH_LAYOUT_TILES_RGBM, each tile followed by its 64-bit blackout mask; `out_bo`
// (nullable) receives blackout_col: the masked pixels as (0, 0, 0, alpha), the others as col.
template <uint32_t BPP> __device__ __forceinline__ typename PixelT<BPP>::T zero_px();
template <> __device__ __forceinline__ uint4 zero_px<16>() { return make_uint4(0u, 0u, 0u, __float_as_uint(1.0f)); }
template <> __device__ __forceinline__ uint2 zero_px<8>() { return make_uint2(0u, 0x3C00u << 16); }
template <> __device__ __forceinline__ uint32_t zero_px<4>() { return 0xFF000000u; }

// P14 (with BPP 8, PLANAR, MASK): BH_LAYOUT_TILES_RGBM14, the 14-bit fp16 channels (86 words per tile:
// r | g << 14 | (b & 0xF) << 28, the bytes (b >> 4) & 0xFF, b's bit-12 and bit-13 words, the mask word).
template <uint32_t BPP, bool PLANAR, bool MASK = false, bool P14 = false>
__global__ void __launch_bounds__(256) tiles_unpack_kernel(const uint32_t* __restrict__ packed, void* __restrict__ out,
                                                           void* __restrict__ out_bo, UnpackGrid u) {
    using P = typename PixelT<BPP>::T;
    static_assert(PLANAR || !MASK, "the mask travels with the planar layout only");
    static_assert(!P14 || (BPP == 8 && PLANAR && MASK), "RGBM14 is an RGBA16F mask layout");
    // 32-bit words per packed tile
    constexpr uint32_t TW = P14 ? 86u : PLANAR ? 12u * BPP + (MASK ? 2u : 0u) : 16u * BPP;
    static_assert(TW % 2u == 0u, "packed tiles are whole 8-byte words");
    constexpr uint32_t TD = TW / 2u;                                // 8-byte words per packed tile
    constexpr uint32_t PER = (UNPACK_SPAN * TD + 255u) / 256u;      // staged words per thread
    __shared__ uint2 lds2[UNPACK_SPAN * TD];
    const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds2);
    __shared__ uint64_t gsrc[UNPACK_SPAN];  // packed tile of each output tile of the span
    const uint32_t tx0 = blockIdx.x * UNPACK_SPAN;
    const uint32_t tiles_y = (u.height + 7u) / 8u;
    const uint32_t span = min(UNPACK_SPAN, u.tiles_x - tx0);       // tiles of the span inside the frame
    const uint2* src = reinterpret_cast<const uint2*>(packed);
    for (uint32_t ty = blockIdx.y; ty < tiles_y; ty += gridDim.y) {  // grid-stride over tile rows
    __syncthreads();  // the previous row's LDS reads are done
    if (threadIdx.x < span) {
        uint32_t k, t;
        if (u.tile_loc) {
            const uint32_t v = u.tile_loc[(size_t)ty * u.tiles_x + tx0 + threadIdx.x];
            k = v >> 24;
            t = v & 0xFFFFFFu;
        } else {
            t = shard_tile_index(tx0 + threadIdx.x, ty, u.tiles_x, u.shard_count, &k);
        }
        gsrc[threadIdx.x] = ((uint64_t)k * u.stride_tiles + t) * TD;
    }
    __syncthreads();
    // Stage the span's packed tiles: consecutive threads take consecutive 8-byte words of a tile, and
    // a shard's tiles of one row are consecutive in its buffer, so each shard's share of the span is
    // one coalesced run.  Every load is issued before the first LDS store (PER loads in flight per
    // thread instead of one tile's worth per wave at a time).
    uint2 v[PER];
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
        const uint32_t i = threadIdx.x + 256u * q, j = i / TD;
        if (j < span) v[q] = src[gsrc[j] + (i - j * TD)];
    }
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
        const uint32_t i = threadIdx.x + 256u * q;
        if (i / TD < span) lds2[i] = v[q];
    }
    __syncthreads();
    const uint32_t x = threadIdx.x, px = tx0 * 8u + x;
    if (px >= u.width) continue;  // no barrier below: lanes past the frame just skip the stores
    const uint32_t* tile = lds + (x >> 3) * TW;
    for (uint32_t r = 0; r < 8u; ++r) {
        const uint32_t py = ty * 8u + r;
        if (py >= u.height) break;
        const uint32_t e = (x & 7u) + 8u * r;  // pixel inside the tile
        P v;
        if constexpr (P14) {
            const uint32_t w = tile[e], hb = (uint32_t)reinterpret_cast<const uint8_t*>(tile + 64)[e];
            const uint32_t b12 = (tile[80u + (e >> 5)] >> (e & 31u)) & 1u, b13 = (tile[82u + (e >> 5)] >> (e & 31u)) & 1u;
            const uint32_t b = (w >> 28) | (hb << 4) | (b12 << 12) | (b13 << 13);
            v = make_uint2((w & 0x3FFFu) | (((w >> 14) & 0x3FFFu) << 16), b | (0x3C00u << 16));
        } else if constexpr (!PLANAR) {
            v = reinterpret_cast<const P*>(tile)[e];
        } else if constexpr (BPP == 16) {  // RGBA32F
            const float* c = reinterpret_cast<const float*>(tile);
            v = make_uint4(__float_as_uint(c[e]), __float_as_uint(c[64 + e]), __float_as_uint(c[128 + e]),
                           __float_as_uint(1.0f));
        } else if constexpr (BPP == 8) {   // RGBA16F
            const uint16_t* c = reinterpret_cast<const uint16_t*>(tile);
            v = make_uint2(c[e] | ((uint32_t)c[64 + e] << 16), c[128 + e] | (0x3C00u << 16));
        } else {                           // BGRA8
            const uint8_t* c = reinterpret_cast<const uint8_t*>(tile);
            v = c[e] | ((uint32_t)c[64 + e] << 8) | ((uint32_t)c[128 + e] << 16) | 0xFF000000u;
        }
        reinterpret_cast<P*>(out)[(size_t)py * u.width + px] = v;
        if constexpr (MASK) {
            if (out_bo) {
                const uint32_t mw = tile[(P14 ? 84u : 12u * BPP) + (e >> 5)];  // the mask word's half holding bit e
                reinterpret_cast<P*>(out_bo)[(size_t)py * u.width + px] = ((mw >> (e & 31u)) & 1u) ? zero_px<BPP>() : v;
            }
        }
    }
    }
}

// Counting sort of the dispatch order by the previous frame's per-tile cost (cost_bucket), one
// kernel: the bucket histogram was accumulated by the march kernel that wrote the costs
// (MarchArgs::order_tot).  A block of ORDER_THREADS threads takes ORDER_PER_BLOCK consecutive
// dispatch slots (each wave a contiguous run of ORDER_PER_WAVE, visited in centre-out order); ranks
// inside a wave come from per-bucket ballots (no LDS atomics), the block's per-wave counts are
// prefix-summed in LDS, and the block reserves its range of every bucket with one returning global
// atomic per bucket.  Ties therefore keep the centre-out order inside a block.  counters: [0..B-1)
// the histogram (the last bucket is the remainder), [B..2B) cursors, [2B] the block ticket; the last
// block to finish zeroes them all, so they are zero again before the next march kernel accumulates
// (graph replay needs no memset node).  (One tile per thread with an LDS atomic per tile and 512
// blocks' global atomics on the same 6 words took 22.8 us per frame; this form ~4 us.)
constexpr uint32_t ORDER_THREADS = 1024;
constexpr uint32_t ORDER_WAVES = ORDER_THREADS / 64u;
constexpr uint32_t ORDER_PER_LANE = 4;
constexpr uint32_t ORDER_PER_WAVE = 64u * ORDER_PER_LANE;
constexpr uint32_t ORDER_PER_BLOCK = ORDER_THREADS * ORDER_PER_LANE;

__global__ void __launch_bounds__(ORDER_THREADS) order_scatter_kernel(const uint8_t* __restrict__ cost, uint32_t n,
                                                                      uint32_t L, uint32_t c, uint32_t* counters,
                                                                      uint32_t* __restrict__ order) {
    __shared__ uint32_t woff[ORDER_WAVES][ORDER_BUCKETS];  // per-wave counts, then offsets in the block
    __shared__ uint32_t base[ORDER_BUCKETS], ticket;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t s0 = blockIdx.x * ORDER_PER_BLOCK + w * ORDER_PER_WAVE + lane;
    uint32_t t[ORDER_PER_LANE], b[ORDER_PER_LANE], r[ORDER_PER_LANE];
    uint32_t cnt[ORDER_BUCKETS];
#pragma unroll
    for (uint32_t q = 0; q < ORDER_BUCKETS; ++q) cnt[q] = 0;
#pragma unroll
    for (uint32_t j = 0; j < ORDER_PER_LANE; ++j) {
        const uint32_t slot = s0 + 64u * j;
        t[j] = slot < n ? centre_out(slot, n, L, c) : 0u;
        b[j] = slot < n ? cost_bucket(cost[t[j]]) : ORDER_BUCKETS;
        r[j] = 0;
#pragma unroll
        for (uint32_t q = 0; q < ORDER_BUCKETS; ++q) {
            const uint64_t m = __ballot(b[j] == q);
            if (b[j] == q)
                r[j] = cnt[q] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            cnt[q] += (uint32_t)__popcll(m);
        }
    }
    if (lane < ORDER_BUCKETS) {
        uint32_t v = 0;
#pragma unroll
        for (uint32_t q = 0; q < ORDER_BUCKETS; ++q) v = lane == q ? cnt[q] : v;
        woff[w][lane] = v;
    }
    __syncthreads();
    if (threadIdx.x < ORDER_BUCKETS) {
        const uint32_t q = threadIdx.x;
        uint32_t tot = 0;
        for (uint32_t v = 0; v < ORDER_WAVES; ++v) {  // exclusive prefix over the block's waves
            const uint32_t x = woff[v][q];
            woff[v][q] = tot;
            tot += x;
        }
        uint32_t off = 0;  // start of bucket q in the order: the histogram's earlier buckets
#pragma unroll
        for (uint32_t j = 0; j < ORDER_BUCKETS - 1u; ++j) off += j < q ? counters[j] : 0u;
        base[q] = tot ? off + atomicAdd(&counters[ORDER_BUCKETS + q], tot) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < ORDER_PER_LANE; ++j)
        if (b[j] < ORDER_BUCKETS) {
            const uint32_t pos = base[b[j]] + woff[w][b[j]] + r[j];
            if (pos < n) order[pos] = t[j];  // defensive: a histogram that disagrees with the costs
        }
    if (threadIdx.x == 0) {
        __threadfence();
        ticket = atomicAdd(&counters[2 * ORDER_BUCKETS], 1u);
    }
    __syncthreads();
    if (ticket == gridDim.x - 1u && threadIdx.x <= 2u * ORDER_BUCKETS) {
        __threadfence();
        atomicExch(&counters[threadIdx.x], 0u);
    }
}

}  // namespace bh

extern "C" __attribute__((visibility("hidden"))) int bh_launch_build_order(const uint8_t* cost, uint32_t n,
                                                                         uint32_t L, uint32_t c,
                                                                         uint32_t* counters, uint32_t* order,
                                                                         hipStream_t s) {
    if (n == 0) return 0;
    const uint32_t blocks = (n + bh::ORDER_PER_BLOCK - 1u) / bh::ORDER_PER_BLOCK;
    hipLaunchKernelGGL(bh::order_scatter_kernel, dim3(blocks), dim3(bh::ORDER_THREADS), 0, s, cost, n, L, c, counters,
                       order);
    return (int)hipGetLastError();
}

static void unpack_launch_shape(uint32_t width, uint32_t height, uint32_t shard_count, uint64_t stride_tiles,
                                uint32_t rows_in_flight, bh::UnpackGrid* u, dim3* grid) {
    u->width = width; u->height = height; u->tiles_x = (width + 7u) / 8u; u->shard_count = shard_count;
    u->stride_tiles = stride_tiles;
    u->tile_loc = nullptr;
    const uint32_t tiles_y = (height + 7u) / 8u;
    // rows_in_flight tile rows per grid pass (0: all), the kernel grid-strides over the rest
    *grid = dim3((u->tiles_x + bh::UNPACK_SPAN - 1u) / bh::UNPACK_SPAN,
                 rows_in_flight && rows_in_flight < tiles_y ? rows_in_flight : tiles_y);
}

template <bool PLANAR, bool MASK>
static int unpack_launch(const void* packed, void* out, void* out_bo, uint32_t width, uint32_t height,
                         uint32_t shard_count, uint64_t stride_tiles, uint32_t bpp, uint32_t rows_in_flight,
                         hipStream_t s, const uint32_t* tile_loc = nullptr, bool p14 = false) {
    bh::UnpackGrid u;
    dim3 grid, block(256);
    unpack_launch_shape(width, height, shard_count, stride_tiles, rows_in_flight, &u, &grid);
    u.tile_loc = tile_loc;
    const uint32_t* p = static_cast<const uint32_t*>(packed);
    if constexpr (PLANAR && MASK) {
        if (p14) {
            if (bpp != 8u) return (int)hipErrorInvalidValue;
            hipLaunchKernelGGL((bh::tiles_unpack_kernel<8, true, true, true>), grid, block, 0, s, p, out, out_bo, u);
            return (int)hipGetLastError();
        }
    }
    switch (bpp) {
        case 16: hipLaunchKernelGGL((bh::tiles_unpack_kernel<16, PLANAR, MASK>), grid, block, 0, s, p, out, out_bo, u); break;
        case 8: hipLaunchKernelGGL((bh::tiles_unpack_kernel<8, PLANAR, MASK>), grid, block, 0, s, p, out, out_bo, u); break;
        case 4: hipLaunchKernelGGL((bh::tiles_unpack_kernel<4, PLANAR, MASK>), grid, block, 0, s, p, out, out_bo, u); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

static uint32_t format_bpp(uint32_t format) {
    return format == BH_OUT_RGBA32F ? 16u : format == BH_OUT_RGBA16F ? 8u : format == BH_OUT_BGRA8_SRGB ? 4u : 0u;
}

extern "C" __attribute__((visibility("hidden"))) int bh_launch_tiles_unpack(const void* packed, void* out, uint32_t width, uint32_t height,
                                      uint32_t shard_count, uint64_t stride_tiles, uint32_t bpp,
                                      hipStream_t s) {
    return unpack_launch<false, false>(packed, out, nullptr, width, height, shard_count, stride_tiles, bpp, 0u, s);
}

extern "C" __attribute__((visibility("hidden"))) int bh_launch_tiles_unpack_rgb(const void* packed, void* out, uint32_t width,
                                                                              uint32_t height, uint32_t shard_count,
                                                                              uint64_t stride_tiles, uint32_t format,
                                                                              uint32_t rows_in_flight, hipStream_t s) {
    return unpack_launch<true, false>(packed, out, nullptr, width, height, shard_count, stride_tiles, format_bpp(format),
                                      rows_in_flight, s);
}

extern "C" __attribute__((visibility("hidden"))) int bh_launch_tiles_unpack_rgbm(const void* packed, void* out, void* out_bo,
                                                                               uint32_t width, uint32_t height,
                                                                               uint32_t shard_count, uint64_t stride_tiles,
                                                                               const uint32_t* tile_loc,
                                                                               uint32_t format, uint32_t rows_in_flight,
                                                                               hipStream_t s) {
    return unpack_launch<true, true>(packed, out, out_bo, width, height, shard_count, stride_tiles,
                                     format_bpp(format & 0xFFu), rows_in_flight, s, tile_loc,
                                     (format & BH_UNPACK_RGBM14) != 0u);
}
