// Lane kernel instantiations m = 33..48 (see benor_lane.h); split so the
// unrolled instantiations build in parallel.
#include "benor_lane.h"

namespace benor {
template hipError_t launch_lane_m<33>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<34>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<35>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<36>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<37>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<38>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<39>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<40>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<41>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<42>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<43>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<44>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<45>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<46>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<47>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<48>(const KParams &, int, hipStream_t);
}  // namespace benor
