// Matrix-core kernel instantiations W = 11..13 (benor_mfma.h: KIND 0..2 x both
// tile parities each), split over four units so the unrolled instantiations
// build in parallel.
#include "benor_mfma.h"

namespace benor {
template hipError_t launch_mfma<11>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<12>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<13>(const KParams &, int, hipStream_t);
}  // namespace benor
