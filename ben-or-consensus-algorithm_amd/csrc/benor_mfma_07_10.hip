// Matrix-core kernel instantiations W = 7..10 (benor_mfma.h: KIND 0..2 x both
// tile parities each), split over four units so the unrolled instantiations
// build in parallel.
#include "benor_mfma.h"

namespace benor {
template hipError_t launch_mfma<7>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<8>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<9>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<10>(const KParams &, int, hipStream_t);
}  // namespace benor
