// bh_tiles.hip — scatter gathered tile-packed shards back into a row-major frame (rank 0 after the
// RCCL gather).  Pure byte movement: one lane per pixel, 16/8/4-byte moves.
#include "bh_common.hpp"

namespace bh {

// Packed tile g (shard-major, each shard padded to stride_tiles) -> its pixel for this lane; false
// for padding tiles and pixels outside the frame.
__device__ __forceinline__ bool unpack_pixel(uint64_t g, uint32_t width, uint32_t height, uint32_t tiles_x,
                                             uint32_t shard_count, uint64_t stride_tiles, uint32_t* px,
                                             uint32_t* py) {
    const uint32_t shard = (uint32_t)(g / stride_tiles);
    const uint32_t t = (uint32_t)(g - (uint64_t)shard * stride_tiles);
    const uint32_t tiles_y = (height + 7u) / 8u;
    if (t >= shard_tile_count(tiles_x, tiles_y, shard, shard_count)) return false;  // padding tiles
    uint32_t tx, ty;
    shard_tile_coords(t, tiles_x, shard, shard_count, &tx, &ty);
    const uint32_t lane = threadIdx.x & 63u;
    *px = tx * 8u + (lane & 7u);
    *py = ty * 8u + (lane >> 3);
    return *px < width && *py < height;
}

template <typename T>
__global__ void __launch_bounds__(256) tiles_unpack_kernel(const T* __restrict__ packed, T* __restrict__ out,
                                                           uint32_t width, uint32_t height, uint32_t tiles_x,
                                                           uint32_t shard_count, uint64_t stride_tiles,
                                                           uint64_t total_tiles) {
    // one wave = one packed tile; consecutive waves walk shard 0's tiles, then shard 1's, ...
    const uint64_t g = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    uint32_t px, py;
    if (g >= total_tiles || !unpack_pixel(g, width, height, tiles_x, shard_count, stride_tiles, &px, &py)) return;
    out[(size_t)py * width + px] = packed[g * 64u + (threadIdx.x & 63u)];
}

// BH_LAYOUT_TILES_RGB: three 64-element channel planes per tile -> RGBA/BGRA texels, alpha restored.
template <uint32_t FMT>
__global__ void __launch_bounds__(256) tiles_unpack_rgb_kernel(const void* __restrict__ packed, void* __restrict__ out,
                                                               uint32_t width, uint32_t height, uint32_t tiles_x,
                                                               uint32_t shard_count, uint64_t stride_tiles,
                                                               uint64_t total_tiles) {
    const uint64_t g = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    uint32_t px, py;
    if (g >= total_tiles || !unpack_pixel(g, width, height, tiles_x, shard_count, stride_tiles, &px, &py)) return;
    const size_t o = g * 192u + (threadIdx.x & 63u), q = (size_t)py * width + px;
    if constexpr (FMT == BH_OUT_RGBA32F) {
        const float* p = reinterpret_cast<const float*>(packed) + o;
        reinterpret_cast<float4*>(out)[q] = make_float4(p[0], p[64], p[128], 1.0f);
    } else if constexpr (FMT == BH_OUT_RGBA16F) {
        const uint16_t* p = reinterpret_cast<const uint16_t*>(packed) + o;
        reinterpret_cast<uint2*>(out)[q] = make_uint2(p[0] | ((uint32_t)p[64] << 16), p[128] | (0x3C00u << 16));
    } else {
        const uint8_t* p = reinterpret_cast<const uint8_t*>(packed) + o;
        reinterpret_cast<uint32_t*>(out)[q] = p[0] | ((uint32_t)p[64] << 8) | ((uint32_t)p[128] << 16) | 0xFF000000u;
    }
}

// Counting sort of the dispatch order by the previous frame's per-tile cost (cost_bucket), one
// kernel: the bucket histogram was accumulated by the march kernel that wrote the costs
// (MarchArgs::order_tot), so each block only reserves its bucket ranges (one returning atomic per
// bucket, issued in parallel) and scatters.  Slots are visited in centre-out order, so ties keep
// (roughly) the centre-out order.  counters: [0..B-1) the histogram (the last bucket is the
// remainder), [B..2B) cursors, [2B] the block ticket; the last block to finish zeroes them all, so
// they are zero again before the next march kernel accumulates (graph replay needs no memset node).
__global__ void __launch_bounds__(256) order_scatter_kernel(const uint8_t* __restrict__ cost, uint32_t n,
                                                          uint32_t L, uint32_t c, uint32_t* counters,
                                                          uint32_t* __restrict__ order) {
    __shared__ uint32_t hist[ORDER_BUCKETS], base[ORDER_BUCKETS], ticket;
    if (threadIdx.x < ORDER_BUCKETS) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t t = 0, b = 0, k = 0;
    if (i < n) {
        t = centre_out(i, n, L, c);
        b = cost_bucket(cost[t]);
        k = atomicAdd(&hist[b], 1u);
    }
    __syncthreads();
    if (threadIdx.x < ORDER_BUCKETS && hist[threadIdx.x]) {
        uint32_t off = 0;
#pragma unroll
        for (uint32_t j = 0; j < ORDER_BUCKETS - 1u; ++j) off += j < threadIdx.x ? counters[j] : 0u;
        base[threadIdx.x] = off + atomicAdd(&counters[ORDER_BUCKETS + threadIdx.x], hist[threadIdx.x]);
    }
    __syncthreads();
    if (i < n) order[base[b] + k] = t;
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
    const uint32_t blocks = (n + 255u) / 256u;
    hipLaunchKernelGGL(bh::order_scatter_kernel, dim3(blocks), dim3(256), 0, s, cost, n, L, c, counters, order);
    return (int)hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) int bh_launch_tiles_unpack(const void* packed, void* out, uint32_t width, uint32_t height,
                                      uint32_t shard_count, uint64_t stride_tiles, uint32_t bpp,
                                      hipStream_t s) {
    const uint32_t tiles_x = (width + 7u) / 8u;
    const uint64_t total = stride_tiles * shard_count;
    const uint64_t blocks = (total + 3u) / 4u;
    if (blocks == 0) return 0;
    if (blocks > 0x7fffffffull) return (int)hipErrorInvalidValue;
    dim3 grid((uint32_t)blocks), block(256);
    switch (bpp) {
        case 16: hipLaunchKernelGGL(bh::tiles_unpack_kernel<uint4>, grid, block, 0, s, (const uint4*)packed, (uint4*)out, width, height, tiles_x, shard_count, stride_tiles, total); break;
        case 8: hipLaunchKernelGGL(bh::tiles_unpack_kernel<uint2>, grid, block, 0, s, (const uint2*)packed, (uint2*)out, width, height, tiles_x, shard_count, stride_tiles, total); break;
        case 4: hipLaunchKernelGGL(bh::tiles_unpack_kernel<uint32_t>, grid, block, 0, s, (const uint32_t*)packed, (uint32_t*)out, width, height, tiles_x, shard_count, stride_tiles, total); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) int bh_launch_tiles_unpack_rgb(const void* packed, void* out, uint32_t width,
                                                                              uint32_t height, uint32_t shard_count,
                                                                              uint64_t stride_tiles, uint32_t format,
                                                                              hipStream_t s) {
    const uint32_t tiles_x = (width + 7u) / 8u;
    const uint64_t total = stride_tiles * shard_count;
    const uint64_t blocks = (total + 3u) / 4u;
    if (blocks == 0) return 0;
    if (blocks > 0x7fffffffull) return (int)hipErrorInvalidValue;
    dim3 grid((uint32_t)blocks), block(256);
    switch (format) {
        case BH_OUT_RGBA32F: hipLaunchKernelGGL(bh::tiles_unpack_rgb_kernel<BH_OUT_RGBA32F>, grid, block, 0, s, packed, out, width, height, tiles_x, shard_count, stride_tiles, total); break;
        case BH_OUT_RGBA16F: hipLaunchKernelGGL(bh::tiles_unpack_rgb_kernel<BH_OUT_RGBA16F>, grid, block, 0, s, packed, out, width, height, tiles_x, shard_count, stride_tiles, total); break;
        case BH_OUT_BGRA8_SRGB: hipLaunchKernelGGL(bh::tiles_unpack_rgb_kernel<BH_OUT_BGRA8_SRGB>, grid, block, 0, s, packed, out, width, height, tiles_x, shard_count, stride_tiles, total); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}
