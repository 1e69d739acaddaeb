// The exact march kernels built WITH machine scheduling (see bh_march_exact.hip): the variant for
// latency-bound frames, whose time is set by the serial step chain of a few long-running waves; its
// tail loop runs the packed-FP32 step (bh_march.hpp, step_tail).
#define BH_NS exact_lat
#define BH_TAIL_PACKED 1
#define BH_EXACT_LAUNCH bh_launch_march_exact_lat
#define BH_EXACT_BLOCKS bh_march_blocks_per_cu_exact_lat
#include "bh_march_exact.hip"
