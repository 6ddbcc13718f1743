// Lane kernel instantiations m = 1..32 (see benor_lane.h); split so the
// unrolled instantiations build in parallel.
#include "benor_lane.h"

namespace benor {
template hipError_t launch_lane_m<1>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<2>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<3>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<4>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<5>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<6>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<7>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<8>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<9>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<10>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<11>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<12>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<13>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<14>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<15>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<16>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<17>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<18>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<19>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<20>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<21>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<22>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<23>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<24>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<25>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<26>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<27>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<28>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<29>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<30>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<31>(const KParams &, int, hipStream_t);
template hipError_t launch_lane_m<32>(const KParams &, int, hipStream_t);
}  // namespace benor
