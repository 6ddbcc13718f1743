// Lane kernel instantiations m = 49..64 (see benor_lane.h); split so the
// unrolled instantiations build in parallel.
#include "benor_lane.h"

namespace benor {
template hipError_t launch_lane_m<49>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<50>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<51>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<52>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<53>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<54>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<55>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<56>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<57>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<58>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<59>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<60>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<61>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<62>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<63>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<64>(const KParams &, int, hipStream_t);
}  // namespace benor
