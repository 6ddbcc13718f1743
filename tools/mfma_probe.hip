// mfma_probe.hip -- gfx950 matrix-core probe for the vote-count formulation:
// (1) which lanes' B-operand data sums into which accumulator column, for
//     v_mfma_scale_f32_16x16x128_f8f6f4 (fp4 e2m1 operands) and
//     v_mfma_i32_16x16x64_i8, with A = all ones and random B (exact integers);
// (2) back-to-back issue rate of both with several waves per SIMD, alone and
//     with VALU filler between MFMAs.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o tools/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void layout_fp4(const int *b, float *d) {
  const int l = threadIdx.x;
  v8i A, B;
  for (int i = 0; i < 8; ++i) { A[i] = 0x22222222; B[i] = b[l * 8 + i]; }   // e2m1 1.0 = 0b0010
  v4f c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A, B, c, 4, 4, 0, 127, 0, 127);
  for (int i = 0; i < 4; ++i) d[l * 4 + i] = c[i];
}

__global__ void layout_i8(const int *b, int *d) {
  const int l = threadIdx.x;
  v4i A, B;
  for (int i = 0; i < 4; ++i) { A[i] = 0x01010101; B[i] = b[l * 4 + i]; }
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) d[l * 4 + i] = c[i];
}

template <int NACC, int FILL>
__global__ void __launch_bounds__(256) rate_fp4(int iters, float *out) {
  const int l = threadIdx.x & 63;
  v8i A, B;
  for (int i = 0; i < 8; ++i) { A[i] = 0x22222222 ^ (l & 1); B[i] = 0x02020202 + l; }
  v4f acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = v4f{(float)j, 0.f, 0.f, 0.f};
  uint32_t f = l;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) {
      acc[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A, B, acc[j], 4, 4, 0, 127, 0, 127);
#pragma unroll
      for (int q = 0; q < FILL; ++q) asm volatile("v_xad_u32 %0, %0, %1, 7" : "+v"(f) : "v"(l));
    }
  }
  float s = (float)f;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC, int FILL>
__global__ void __launch_bounds__(256) rate_i8(int iters, int *out) {
  const int l = threadIdx.x & 63;
  v4i A, B;
  for (int i = 0; i < 4; ++i) { A[i] = 0x01010101 ^ (l & 1); B[i] = 0x01000100 + l; }
  v4i acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = v4i{j, 0, 0, 0};
  uint32_t f = l;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) {
      acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B, acc[j], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < FILL; ++q) asm volatile("v_xad_u32 %0, %0, %1, 7" : "+v"(f) : "v"(l));
    }
  }
  int s = (int)f;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef short v8s __attribute__((ext_vector_type(8)));

template <int NACC>
__global__ void __launch_bounds__(256) rate_fp4_32(int iters, float *out) {
  const int l = threadIdx.x & 63;
  v8i A, B;
  for (int i = 0; i < 8; ++i) { A[i] = 0x22222222 ^ (l & 1); B[i] = 0x02020202 + l; }
  v16f acc[NACC];
  for (int j = 0; j < NACC; ++j) { acc[j] = v16f{}; acc[j][0] = (float)j; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NACC; ++j)
      acc[j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, acc[j], 4, 4, 0, 127, 0, 127);
  }
  float s = 0.f;
  for (int j = 0; j < NACC; ++j) for (int i = 0; i < 16; ++i) s += acc[j][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ void __launch_bounds__(256) rate_i8_32(int iters, int *out) {
  const int l = threadIdx.x & 63;
  v4i A, B;
  for (int i = 0; i < 4; ++i) { A[i] = 0x01010101 ^ (l & 1); B[i] = 0x01000100 + l; }
  v16i acc[NACC];
  for (int j = 0; j < NACC; ++j) { acc[j] = v16i{}; acc[j][0] = j; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, acc[j], 0, 0, 0);
  }
  int s = 0;
  for (int j = 0; j < NACC; ++j) for (int i = 0; i < 16; ++i) s += acc[j][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ void __launch_bounds__(256) rate_bf16(int iters, float *out) {
  const int l = threadIdx.x & 63;
  v8s A, B;
  for (int i = 0; i < 8; ++i) { A[i] = (short)(0x3f80 ^ (l & 1)); B[i] = (short)(0x3f80 + (l & 3)); }
  v4f acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = v4f{(float)j, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B, acc[j], 0, 0, 0);
  }
  float s = 0.f;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static const float kE2M1[8] = {0.f, 0.5f, 1.f, 1.5f, 2.f, 3.f, 4.f, 6.f};

template <typename K, typename T>
static void time_rate(const char *name, K kern, int nacc, int fill, int waves_per_simd, T *out) {
  const int blocks = 256 * waves_per_simd;     // 4 waves per block: waves_per_simd waves on each SIMD
  const int iters = 4000;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, 10, out);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, iters, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double mfma = (double)blocks * 4 * iters * nacc;
  const double per_simd_ns = ms * 1e6 / (mfma / 1024.0);
  printf("{\"probe\": \"%s\", \"nacc\": %d, \"valu_fill\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, "
         "\"ns_per_mfma_per_simd\": %.4f, \"cycles_at_2p4GHz\": %.2f}\n",
         name, nacc, fill, waves_per_simd, ms, per_simd_ns, per_simd_ns * 2.4);
}

int main() {
  srand(12345);
  // ---- layout fp4
  {
    std::vector<int> b(64 * 8);
    std::vector<int> nib(64 * 8 * 8);
    for (int l = 0; l < 64; ++l)
      for (int v = 0; v < 8; ++v) {
        uint32_t w = 0;
        for (int j = 0; j < 8; ++j) {
          const int code = rand() % 8;
          nib[(l * 8 + v) * 8 + j] = code;
          w |= (uint32_t)code << (4 * j);
        }
        b[l * 8 + v] = (int)w;
      }
    int *db; float *dd;
    CK(hipMalloc(&db, b.size() * 4));
    CK(hipMalloc(&dd, 64 * 4 * 4));
    CK(hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(layout_fp4, dim3(1), dim3(64), 0, 0, db, dd);
    std::vector<float> d(256);
    CK(hipMemcpy(d.data(), dd, 256 * 4, hipMemcpyDeviceToHost));
    // hypotheses: column = lane & 15, summing the B data of lanes n, n+16, n+32, n+48 over
    // (a) all 8 VGPRs, (b) the low 4 VGPRs only
    int ok_a = 1, ok_b = 1;
    for (int l = 0; l < 64; ++l) {
      const int n = l & 15;
      double sa = 0, sb = 0;
      for (int g = 0; g < 4; ++g)
        for (int v = 0; v < 8; ++v)
          for (int j = 0; j < 8; ++j) {
            const float x = kE2M1[nib[((n + 16 * g) * 8 + v) * 8 + j]];
            sa += x;
            if (v < 4) sb += x;
          }
      for (int r = 0; r < 4; ++r) {
        if (d[l * 4 + r] != (float)sa) ok_a = 0;
        if (d[l * 4 + r] != (float)sb) ok_b = 0;
      }
    }
    printf("{\"probe\": \"layout_fp4_16x16x128\", \"col_lane_and_15_all8\": %d, \"col_lane_and_15_low4\": %d, "
           "\"lane0\": [%g, %g, %g, %g], \"lane17\": [%g, %g, %g, %g]}\n",
           ok_a, ok_b, d[0], d[1], d[2], d[3], d[68], d[69], d[70], d[71]);
  }
  // ---- layout i8
  {
    std::vector<int> b(64 * 4);
    std::vector<int> by(64 * 16);
    for (int l = 0; l < 64; ++l)
      for (int v = 0; v < 4; ++v) {
        uint32_t w = 0;
        for (int j = 0; j < 4; ++j) {
          const int x = (rand() % 5) - 2;
          by[(l * 4 + v) * 4 + j] = x;
          w |= (uint32_t)(uint8_t)(int8_t)x << (8 * j);
        }
        b[l * 4 + v] = (int)w;
      }
    int *db, *dd;
    CK(hipMalloc(&db, b.size() * 4));
    CK(hipMalloc(&dd, 256 * 4));
    CK(hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(layout_i8, dim3(1), dim3(64), 0, 0, db, dd);
    std::vector<int> d(256);
    CK(hipMemcpy(d.data(), dd, 256 * 4, hipMemcpyDeviceToHost));
    int ok = 1;
    for (int l = 0; l < 64; ++l) {
      const int n = l & 15;
      int s = 0;
      for (int g = 0; g < 4; ++g)
        for (int k = 0; k < 16; ++k) s += by[(n + 16 * g) * 16 + k];
      for (int r = 0; r < 4; ++r)
        if (d[l * 4 + r] != s) ok = 0;
    }
    printf("{\"probe\": \"layout_i8_16x16x64\", \"col_lane_and_15\": %d, \"lane0\": [%d, %d, %d, %d]}\n", ok, d[0], d[1],
           d[2], d[3]);
  }
  // ---- rates
  float *of;
  int *oi;
  CK(hipMalloc(&of, 256 * 8 * 256 * 4));
  CK(hipMalloc(&oi, 256 * 8 * 256 * 4));
  for (int w : {1, 2, 4}) {
    time_rate("fp4_16x16x128", rate_fp4<4, 0>, 4, 0, w, of);
    time_rate("i8_16x16x64", rate_i8<4, 0>, 4, 0, w, oi);
  }
  time_rate("bf16_16x16x32", rate_bf16<4>, 4, 0, 2, of);
  time_rate("bf16_16x16x32", rate_bf16<4>, 4, 0, 4, of);
  time_rate("fp4_32x32x64", rate_fp4_32<4>, 4, 0, 2, of);
  time_rate("fp4_32x32x64", rate_fp4_32<2>, 2, 0, 4, of);
  time_rate("i8_32x32x32", rate_i8_32<4>, 4, 0, 2, oi);
  time_rate("i8_32x32x32", rate_i8_32<2>, 2, 0, 4, oi);
  time_rate("fp4_16x16x128", rate_fp4<1, 0>, 1, 0, 1, of);
  time_rate("fp4_16x16x128", rate_fp4<8, 0>, 8, 0, 2, of);
  time_rate("fp4_16x16x128", rate_fp4<4, 1>, 4, 1, 2, of);
  time_rate("fp4_16x16x128", rate_fp4<4, 2>, 4, 2, 2, of);
  time_rate("fp4_16x16x128", rate_fp4<4, 3>, 4, 3, 2, of);
  time_rate("fp4_16x16x128", rate_fp4<4, 4>, 4, 4, 2, of);
  time_rate("fp4_16x16x128", rate_fp4<4, 2>, 4, 2, 4, of);
  time_rate("fp4_16x16x128", rate_fp4<4, 4>, 4, 4, 4, of);
  time_rate("i8_16x16x64", rate_i8<4, 2>, 4, 2, 2, oi);
  time_rate("i8_16x16x64", rate_i8<4, 4>, 4, 4, 2, oi);
  return 0;
}
