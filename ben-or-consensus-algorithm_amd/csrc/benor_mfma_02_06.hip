// Matrix-core kernel instantiations W = 2..6 (benor_mfma.h: KIND 0..2 x both
// tile parities each), split over four units so the unrolled instantiations
// build in parallel.
#include "benor_mfma.h"

namespace benor {
template hipError_t launch_mfma<2>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<3>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<4>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<5>(const KParams &, int, hipStream_t);
template hipError_t launch_mfma<6>(const KParams &, int, hipStream_t);
}  // namespace benor

namespace benor {

// Matrix-core peak probe: the kernel's instruction back-to-back on two
// independent accumulators per wave (tools/mfma_probe.hip: 2-4 waves per SIMD
// reach the issue rate), operands as the kernel's (ones x 0/1 nibbles).
__global__ void __launch_bounds__(256) mfma_peak_kernel(float *sink, int iters) {
  const uint32_t lane = threadIdx.x & 63u;
  mf_v4i a = {0x22222222, 0x22222222, 0x22222222, 0x22222222};
  const mf_v4i b = expand_votes(0x9E3779B9u * (lane + 1u));
  mf_v16f acc0 = {}, acc1 = {};
  for (int i = 0; i < iters; ++i) {
    asm volatile("" : "+v"(a));
    acc0 = mfma_count(a, b, acc0);
    acc1 = mfma_count(a, b, acc1);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += acc0[j] + acc1[j];
  if (s == 1.0f) sink[blockIdx.x] = s;   // never true: keeps the loop
}

hipError_t launch_mfma_peak(float *sink, int grid, int iters, hipStream_t s, double *terms) {
  hipLaunchKernelGGL(mfma_peak_kernel, dim3(grid), dim3(256), 0, s, sink, iters);
  if (terms) *terms = (double)grid * 4.0 * 2.0 * (double)iters * 65536.0;
  return hipGetLastError();
}

}  // namespace benor
