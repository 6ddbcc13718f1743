// mfma32_probe.hip -- issue behaviour of v_mfma_scale_f32_32x32x64_f8f6f4
// (e2m1 operands, the matrix-core kernels' instruction) on gfx950, for the
// configs[2] question of DESIGN §9: how many cycles one wave-level MFMA takes
// per SIMD when
//   * CH independent accumulator chains are interleaved in a wave (CH = 1: every
//     MFMA reads the previous one's result as C, as a receiver tile's K chunks do),
//   * FILL independent VALU instructions follow each MFMA (the sign packing /
//     fold that the kernel interleaves),
//   * NV waves share a SIMD (one-wave workgroups, NV * 4 per CU).
// Prints one JSON line per case: ns and shader-clock cycles per MFMA per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form tools/mfma32_probe.hip -o tools/mfma32_probe
// (the VGPR form, as the product kernels are built)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int CH, int FILL>
__global__ void __launch_bounds__(64) chain_kernel(int iters, float *out, unsigned long long *cyc) {
  const int l = threadIdx.x;
  v8i A, B;
  for (int i = 0; i < 8; ++i) { A[i] = i < 4 ? 0x22222222 : 0; B[i] = i < 4 ? (0x02020202 ^ (l & 1)) : 0; }
  v16f acc[CH];
  for (int j = 0; j < CH; ++j)
    for (int k = 0; k < 16; ++k) acc[j][k] = (float)(j + k);
  uint32_t f[4] = {(uint32_t)l, (uint32_t)l + 1u, (uint32_t)l + 2u, (uint32_t)l + 3u};   // 4 independent filler chains
  const unsigned long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      acc[j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, acc[j], 4, 4, 0, 127, 0, 127);
#pragma unroll
      for (int q = 0; q < FILL; ++q) asm volatile("v_xad_u32 %0, %0, %1, 7" : "+v"(f[q & 3]) : "v"(l));
    }
  }
  const unsigned long long t1 = clock64();
  float s = (float)(f[0] ^ f[1] ^ f[2] ^ f[3]);
  for (int j = 0; j < CH; ++j)
    for (int k = 0; k < 16; ++k) s += acc[j][k];
  out[blockIdx.x * 64 + l] = s;
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CH, int FILL>
static void run(int nv, int iters, float *out, unsigned long long *cyc, int cus) {
  const int blocks = cus * 4 * nv;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((chain_kernel<CH, FILL>), dim3(blocks), dim3(64), 0, 0, 16, out, cyc);   // warm-up
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL((chain_kernel<CH, FILL>), dim3(blocks), dim3(64), 0, 0, iters, out, cyc);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long *h = (unsigned long long *)malloc(sizeof(unsigned long long) * blocks);
  CK(hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost));
  double avg = 0;
  for (int i = 0; i < blocks; ++i) avg += (double)h[i];
  avg /= blocks;
  free(h);
  const double mfma_per_simd = (double)nv * iters * CH;   // NV waves per SIMD
  printf("{\"chains\": %d, \"fill_valu\": %d, \"waves_per_simd\": %d, \"ns_per_mfma_per_simd\": %.2f, "
         "\"wave_cycles_per_own_mfma\": %.1f, \"ms\": %.3f}\n",
         CH, FILL, nv, ms * 1e6 / mfma_per_simd, avg / ((double)iters * CH), ms);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float *out;
  unsigned long long *cyc;
  CK(hipMalloc(&out, sizeof(float) * cus * 4 * 8 * 64));
  CK(hipMalloc(&cyc, sizeof(unsigned long long) * cus * 4 * 8));
  const int it = 4000;
  for (int nv : {1, 2, 4}) {
    run<1, 0>(nv, it, out, cyc, cus);
    run<2, 0>(nv, it / 2, out, cyc, cus);
    run<3, 0>(nv, it / 3, out, cyc, cus);
    run<1, 5>(nv, it, out, cyc, cus);
    run<2, 5>(nv, it / 2, out, cyc, cus);
    run<1, 8>(nv, it, out, cyc, cus);
    run<1, 16>(nv, it, out, cyc, cus);
    run<2, 8>(nv, it / 2, out, cyc, cus);
  }
  CK(hipFree(out));
  CK(hipFree(cyc));
  return 0;
}
