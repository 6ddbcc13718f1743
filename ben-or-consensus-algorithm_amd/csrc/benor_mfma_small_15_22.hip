// Packed matrix-core kernel instantiations m = 15..22 (see benor_mfma_small.h); the
// m = 2..32 range is split over four translation units for a parallel build.
#include "benor_mfma_small.h"

namespace benor {
#define BENOR_SMALL(M) template hipError_t launch_mfma_small_m<M>(const KParams &, int, hipStream_t);
BENOR_SMALL(15) BENOR_SMALL(16) BENOR_SMALL(17) BENOR_SMALL(18) BENOR_SMALL(19) BENOR_SMALL(20) BENOR_SMALL(21) BENOR_SMALL(22)
#undef BENOR_SMALL
}  // namespace benor
