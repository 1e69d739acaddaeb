// Fast (production) instantiation of the march kernel.  Built with -ffp-contract=fast and
// -fno-hip-fp32-correctly-rounded-divide-sqrt: hardware rcp/rsq/sqrt, FMA contraction.
#define BH_FAST 1
#define BH_NS fast
#include "bh_march.hpp"

extern "C" __attribute__((visibility("hidden"))) int bh_launch_march_fast(const bh::MarchArgs& a, hipStream_t s) {
    const uint32_t blocks = (a.n_tiles + 3u) / 4u;
    hipLaunchKernelGGL(bh::fast::march_kernel, dim3(blocks), dim3(256), 0, s, a);
    return (int)hipGetLastError();
}
