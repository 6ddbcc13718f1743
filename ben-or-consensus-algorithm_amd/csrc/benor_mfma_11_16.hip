// Matrix-core kernel instantiations W = 11..16 (benor_mfma.h).
#include "benor_mfma.h"

namespace benor {
template hipError_t launch_mfma<11>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<12>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<13>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<14>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<15>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<16>(const KParams &, int, hipStream_t);
}  // namespace benor
