// Packed matrix-core kernel instantiations m = 8..14 (see benor_mfma_small.h); the
// m = 2..32 range is split over four translation units for a parallel build.
#include "benor_mfma_small.h"

namespace benor {
#define BENOR_SMALL(M) template hipError_t launch_mfma_small_m<M>(const KParams &, int, hipStream_t);
BENOR_SMALL(8) BENOR_SMALL(9) BENOR_SMALL(10) BENOR_SMALL(11) BENOR_SMALL(12) BENOR_SMALL(13) BENOR_SMALL(14)
#undef BENOR_SMALL
}  // namespace benor
