// Exact (parity) instantiation of the march kernel.  Built with -ffp-contract=off and the default
// correctly-rounded f32 division/sqrt: same op sequence as oracle/bh_oracle.c (bit-exact parity).
#define BH_FAST 0
#define BH_NS exact
#include "bh_march.hpp"

extern "C" __attribute__((visibility("hidden"))) int bh_launch_march_exact(const bh::MarchArgs& a, hipStream_t s) {
    const uint32_t blocks = (a.n_tiles + 3u) / 4u;
    hipLaunchKernelGGL(bh::exact::march_kernel, dim3(blocks), dim3(256), 0, s, a);
    return (int)hipGetLastError();
}
