// W kernel instantiations W = 2..17 (see benor_w_kernel.h; m <= 64, W = 1, runs in
// the lane kernel, benor_lane.h); split so the
// unrolled instantiations (compile time ~ W^2) build in parallel.
#include "benor_w_kernel.h"

namespace benor {
template hipError_t launch_w<2>(const KParams &, int, hipStream_t);
template hipError_t launch_w<3>(const KParams &, int, hipStream_t);
template hipError_t launch_w<4>(const KParams &, int, hipStream_t);
template hipError_t launch_w<5>(const KParams &, int, hipStream_t);
template hipError_t launch_w<6>(const KParams &, int, hipStream_t);
template hipError_t launch_w<7>(const KParams &, int, hipStream_t);
template hipError_t launch_w<8>(const KParams &, int, hipStream_t);
template hipError_t launch_w<9>(const KParams &, int, hipStream_t);
template hipError_t launch_w<10>(const KParams &, int, hipStream_t);
template hipError_t launch_w<11>(const KParams &, int, hipStream_t);
template hipError_t launch_w<12>(const KParams &, int, hipStream_t);
template hipError_t launch_w<13>(const KParams &, int, hipStream_t);
template hipError_t launch_w<14>(const KParams &, int, hipStream_t);
template hipError_t launch_w<15>(const KParams &, int, hipStream_t);
template hipError_t launch_w<16>(const KParams &, int, hipStream_t);
template hipError_t launch_w<17>(const KParams &, int, hipStream_t);
}  // namespace benor
