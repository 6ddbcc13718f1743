// Item kernel instantiations m = 2..24 (see benor_lane_items.h).
#include "benor_lane_items.h"

namespace benor {
#define BENOR_ITEMS(M) template hipError_t launch_items_m<M>(const KParams &, int, hipStream_t);
BENOR_ITEMS(2) BENOR_ITEMS(3) BENOR_ITEMS(4) BENOR_ITEMS(5) BENOR_ITEMS(6) BENOR_ITEMS(7) BENOR_ITEMS(8)
BENOR_ITEMS(9) BENOR_ITEMS(10) BENOR_ITEMS(11) BENOR_ITEMS(12) BENOR_ITEMS(13) BENOR_ITEMS(14) BENOR_ITEMS(15)
BENOR_ITEMS(16) BENOR_ITEMS(17) BENOR_ITEMS(18) BENOR_ITEMS(19) BENOR_ITEMS(20) BENOR_ITEMS(21) BENOR_ITEMS(22)
BENOR_ITEMS(23) BENOR_ITEMS(24)
#undef BENOR_ITEMS
}  // namespace benor
