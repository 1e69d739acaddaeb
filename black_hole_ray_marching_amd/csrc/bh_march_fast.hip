// Fast (production) instantiation of the march kernel.  Built with -ffp-contract=fast and
// -fno-hip-fp32-correctly-rounded-divide-sqrt: hardware rcp/rsq/sqrt, FMA contraction.
#define BH_FAST 1
#define BH_NS fast
#include "bh_march.hpp"

namespace {
template <uint32_t FMT>
int launch(const bh::MarchArgs& a, uint32_t schedule, uint32_t* counters, uint32_t grid, hipStream_t s) {
    if (schedule == BH_SCHED_TILE) {
        if (a.scene_flags == BH_SCENE_DEFAULT)  // the reference's scene: flags folded at compile time
            bh::fast::launch_tile_schedule<FMT, BH_SCENE_DEFAULT>(a, s);
        else
            bh::fast::launch_tile_schedule<FMT, bh::fast::SF_DYN>(a, s);
    } else if (schedule == BH_SCHED_PAIR) {
        const uint32_t pairs = (a.n_tiles + 1u) / 2u;
        hipLaunchKernelGGL(bh::fast::march_pair_kernel<FMT>, dim3((pairs + 3u) / 4u), dim3(256), 0, s, a);
    } else {
        hipError_t e = hipMemsetAsync(counters, 0, bh::fast::NQ * bh::fast::CTR_STRIDE * sizeof(uint32_t), s);
        if (e != hipSuccess) return (int)e;
        hipLaunchKernelGGL(bh::fast::march_persistent_kernel<FMT>, dim3(grid), dim3(256), 0, s, a, counters);
    }
    return (int)hipGetLastError();
}
}  // namespace

extern "C" __attribute__((visibility("hidden"))) int bh_launch_march_fast(const bh::MarchArgs& a, uint32_t schedule,
                                                                             uint32_t* counters, uint32_t grid,
                                                                             hipStream_t s) {
    switch (a.format) {
        case BH_OUT_RGBA32F: return launch<BH_OUT_RGBA32F>(a, schedule, counters, grid, s);
        case BH_OUT_RGBA16F: return launch<BH_OUT_RGBA16F>(a, schedule, counters, grid, s);
        default: return launch<BH_OUT_BGRA8_SRGB>(a, schedule, counters, grid, s);
    }
}

// Resident 256-thread blocks per CU of the persistent kernel (sizes its grid: every block resident).
extern "C" __attribute__((visibility("hidden"))) int bh_march_blocks_per_cu_fast(void) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, bh::fast::march_persistent_kernel<BH_OUT_BGRA8_SRGB>, 256, 0) != hipSuccess) return 1;
    return n > 0 ? n : 1;
}
