// bh_tiles.hip — scatter gathered tile-packed shards back into a row-major frame (rank 0 after the
// RCCL gather).  Pure byte movement: one lane per pixel, 16/8/4-byte moves.
#include "bh_common.hpp"

namespace bh {

template <typename T>
__global__ void __launch_bounds__(256) tiles_unpack_kernel(const T* __restrict__ packed, T* __restrict__ out,
                                                           uint32_t width, uint32_t height, uint32_t tiles_x,
                                                           uint32_t shard_count, uint64_t stride_tiles,
                                                           uint64_t total_tiles) {
    // one wave = one packed tile; consecutive waves walk shard 0's tiles, then shard 1's, ...
    const uint64_t g = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    if (g >= total_tiles) return;
    const uint32_t shard = (uint32_t)(g / stride_tiles);
    const uint32_t t = (uint32_t)(g - (uint64_t)shard * stride_tiles);
    const uint32_t tiles_y = (height + 7u) / 8u;
    if (t >= shard_tile_count(tiles_x, tiles_y, shard, shard_count)) return;  // padding tiles
    uint32_t tx, ty;
    shard_tile_coords(t, tiles_x, shard, shard_count, &tx, &ty);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t px = tx * 8u + (lane & 7u), py = ty * 8u + (lane >> 3);
    if (px >= width || py >= height) return;
    out[(size_t)py * width + px] = packed[g * 64u + lane];
}

}  // namespace bh

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
