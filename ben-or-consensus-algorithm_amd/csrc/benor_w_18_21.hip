// W kernel instantiations W = 18..21 (see benor_w_kernel.h); split so the
// unrolled instantiations (compile time ~ W^2) build in parallel.
#include "benor_w_kernel.h"

namespace benor {
template hipError_t launch_w<18>(const KParams &, int, hipStream_t);
template hipError_t launch_w<19>(const KParams &, int, hipStream_t);
template hipError_t launch_w<20>(const KParams &, int, hipStream_t);
template hipError_t launch_w<21>(const KParams &, int, hipStream_t);
}  // namespace benor
