// Packed matrix-core kernel instantiations m = 2..7 (see benor_mfma_small.h); the
// m = 2..32 range is split over four translation units for a parallel build.
#include "benor_mfma_small.h"

namespace benor {
#define BENOR_SMALL(M) template hipError_t launch_mfma_small_m<M>(const KParams &, int, hipStream_t);
BENOR_SMALL(2) BENOR_SMALL(3) BENOR_SMALL(4) BENOR_SMALL(5) BENOR_SMALL(6) BENOR_SMALL(7)
#undef BENOR_SMALL
}  // namespace benor
