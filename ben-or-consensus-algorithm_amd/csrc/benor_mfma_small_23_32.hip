// Packed matrix-core kernel instantiations m = 23..32 (see benor_mfma_small.h); the
// m = 2..32 range is split over four translation units for a parallel build.
#include "benor_mfma_small.h"

namespace benor {
#define BENOR_SMALL(M) template hipError_t launch_mfma_small_m<M>(const KParams &, int, hipStream_t);
BENOR_SMALL(23) BENOR_SMALL(24) BENOR_SMALL(25) BENOR_SMALL(26) BENOR_SMALL(27) BENOR_SMALL(28) BENOR_SMALL(29) BENOR_SMALL(30) BENOR_SMALL(31) BENOR_SMALL(32)
#undef BENOR_SMALL
}  // namespace benor
