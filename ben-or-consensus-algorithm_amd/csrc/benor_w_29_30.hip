// W kernel instantiations W = 29..30 (see benor_w_kernel.h); split so the
// unrolled instantiations (compile time ~ W^2) build in parallel.
#include "benor_w_kernel.h"

namespace benor {
template hipError_t launch_w<29>(const KParams &, int, hipStream_t);
template hipError_t launch_w<30>(const KParams &, int, hipStream_t);
}  // namespace benor
