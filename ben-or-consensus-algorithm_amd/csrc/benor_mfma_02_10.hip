// Matrix-core kernel instantiations W = 2..10 (benor_mfma.h), split from
// W = 11..16 so the unrolled instantiations build in parallel.
#include "benor_mfma.h"

namespace benor {
template hipError_t launch_mfma<2>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<3>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<4>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<5>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<6>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<7>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<8>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<9>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<10>(const KParams &, int, hipStream_t);
}  // namespace benor
