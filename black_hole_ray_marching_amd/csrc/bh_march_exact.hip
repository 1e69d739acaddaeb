// Exact (parity) instantiation of the march kernel.  Built with -ffp-contract=off and the default
// correctly-rounded f32 division/sqrt: same op sequence as oracle/bh_oracle.c (bit-exact parity).
//
// Two builds of this file (same source, same arithmetic, different instruction schedules; build.py):
//   bh_march_exact.hip      namespace exact      no machine scheduling: the step in source order, the
//                                                faster issue stream for throughput-bound frames;
//   bh_march_exact_lat.hip  namespace exact_lat  LLVM's machine schedulers: interleaved chains, the
//                                                shorter latency per step of a lone tail wave.
// bh_render picks one per frame (bh_host.cpp, march_variant).
#define BH_FAST 0
#ifndef BH_NS
#define BH_NS exact
#define BH_EXACT_LAUNCH bh_launch_march_exact
#define BH_EXACT_BLOCKS bh_march_blocks_per_cu_exact
#define BH_EXACT_AUX 1
#endif
#include "bh_march.hpp"

namespace {
template <uint32_t FMT>
int launch(const bh::MarchArgs& a, uint32_t schedule, uint32_t* counters, uint32_t grid, hipStream_t s) {
    if (schedule == BH_SCHED_TILE) {
        if (a.scene_flags == BH_SCENE_DEFAULT)  // the reference's scene: flags folded at compile time
            bh::BH_NS::launch_tile_schedule<FMT, BH_SCENE_DEFAULT>(a, s);
        else if (a.scene_flags == 0u)  // no surfaces (BASELINE config 1): the sdf folds to +inf
            bh::BH_NS::launch_tile_schedule<FMT, 0u>(a, s);
        else
            bh::BH_NS::launch_tile_schedule<FMT, bh::BH_NS::SF_DYN>(a, s);
    } else if (schedule == BH_SCHED_PAIR) {
        const uint32_t pairs = (a.n_tiles + 1u) / 2u;
        hipLaunchKernelGGL(bh::BH_NS::march_pair_kernel<FMT>, dim3((pairs + 3u) / 4u), dim3(256), 0, s, a);
    } else {
        hipError_t e = hipMemsetAsync(counters, 0, bh::BH_NS::NQ * bh::BH_NS::CTR_STRIDE * sizeof(uint32_t), s);
        if (e != hipSuccess) return (int)e;
        hipLaunchKernelGGL(bh::BH_NS::march_persistent_kernel<FMT>, dim3(grid), dim3(256), 0, s, a, counters);
    }
    return (int)hipGetLastError();
}
}  // namespace

extern "C" __attribute__((visibility("hidden"))) int BH_EXACT_LAUNCH(const bh::MarchArgs& a, uint32_t schedule,
                                                                             uint32_t* counters, uint32_t grid,
                                                                             hipStream_t s) {
    switch (a.format) {
        case BH_OUT_RGBA32F: return launch<BH_OUT_RGBA32F>(a, schedule, counters, grid, s);
        case BH_OUT_RGBA16F: return launch<BH_OUT_RGBA16F>(a, schedule, counters, grid, s);
        default: return launch<BH_OUT_BGRA8_SRGB>(a, schedule, counters, grid, s);
    }
}

// Resident 256-thread blocks per CU of the persistent kernel (sizes its grid: every block resident).
extern "C" __attribute__((visibility("hidden"))) int BH_EXACT_BLOCKS(void) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, bh::BH_NS::march_persistent_kernel<BH_OUT_BGRA8_SRGB>, 256, 0) != hipSuccess) return 1;
    return n > 0 ? n : 1;
}

#if defined(BH_DIAG_SLOW) && defined(BH_EXACT_AUX)
// diagnostics build only: read and reset the fallback counters
extern "C" int bh_diag_slow_counts(uint32_t* lane_steps, uint32_t* wave_steps) {
    uint32_t z = 0;
    if (hipMemcpyFromSymbol(lane_steps, HIP_SYMBOL(bh::BH_NS::g_diag_slow_lane_steps), 4) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(wave_steps, HIP_SYMBOL(bh::BH_NS::g_diag_slow_wave_steps), 4) != hipSuccess) return -1;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(bh::BH_NS::g_diag_slow_lane_steps), &z, 4);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(bh::BH_NS::g_diag_slow_wave_steps), &z, 4);
    return 0;
}
// and the root-free step's counters: wave-steps that skipped the SDF roots (far field included), all
// wave-steps, far-field wave-steps
extern "C" int bh_diag_far_count(uint32_t* far_wave_steps) {
    uint32_t z = 0;
    if (hipMemcpyFromSymbol(far_wave_steps, HIP_SYMBOL(bh::BH_NS::g_diag_far_wave_steps), 4) != hipSuccess) return -1;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(bh::BH_NS::g_diag_far_wave_steps), &z, 4);
    return 0;
}
extern "C" int bh_diag_skip_counts(uint32_t* skip_wave_steps, uint32_t* all_wave_steps) {
    uint32_t z = 0;
    if (hipMemcpyFromSymbol(skip_wave_steps, HIP_SYMBOL(bh::BH_NS::g_diag_skip_wave_steps), 4) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(all_wave_steps, HIP_SYMBOL(bh::BH_NS::g_diag_all_wave_steps), 4) != hipSuccess) return -1;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(bh::BH_NS::g_diag_skip_wave_steps), &z, 4);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(bh::BH_NS::g_diag_all_wave_steps), &z, 4);
    return 0;
}
#endif
