// W kernel instantiations W = 22..24 (see benor_w_kernel.h); split so the
// unrolled instantiations (compile time ~ W^2) build in parallel.
#include "benor_w_kernel.h"

namespace benor {
template hipError_t launch_w<22>(const KParams &, int, hipStream_t);
template hipError_t launch_w<23>(const KParams &, int, hipStream_t);
template hipError_t launch_w<24>(const KParams &, int, hipStream_t);
}  // namespace benor
