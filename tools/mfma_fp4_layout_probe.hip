// Checks the K pairing of v_mfma_scale_f32_32x32x64_f8f6f4 with e2m1 (fp4)
// operands on gfx950: A lane (row r, half h) nibble n of VGPR v and B lane
// (col c, half h) nibble n of VGPR v must multiply the same k.  The packed
// small-network kernel (benor_mfma_small.h) builds a block-diagonal A on this
// assumption.  For every K position p = (h, v, n): A row 0 is one-hot at p,
// B column c is one-hot at position c (c < 32) or c + 32 (second pass); the
// result row 0 must be one-hot at the column holding p.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_fp4_layout_probe.hip -o /tmp/fp4probe && /tmp/fp4probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void probe(int p, int pass, float *out) {
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  v4i a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
  const int ph = p >> 5, pv = (p >> 3) & 3, pn = p & 7;
  if (r == 0 && h == ph) a[pv] = 0x2 << (4 * pn);                      // A[0][p] = 1.0
  const int q = r + 32 * pass;                                          // column r holds position q
  if (h == (q >> 5)) b[(q >> 3) & 3] = 0x2 << (4 * (q & 7));           // B[q][r] = 1.0
  v16f c = {};
  const v8i a8 = __builtin_shufflevector(a, a, 0, 1, 2, 3, -1, -1, -1, -1);
  const v8i b8 = __builtin_shufflevector(b, b, 0, 1, 2, 3, -1, -1, -1, -1);
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, 127, 0, 127);
  // row 0 lives in register j = 0 of lanes 0..31 (row = (j&3) + 8(j>>2) + 4h)
  if (h == 0) out[r] = c[0];
}

int main() {
  float *d;
  hipMalloc(&d, 32 * sizeof(float));
  int bad = 0;
  for (int p = 0; p < 64; ++p) {
    for (int pass = 0; pass < 2; ++pass) {
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, p, pass, d);
      float o[32];
      hipMemcpy(o, d, sizeof o, hipMemcpyDeviceToHost);
      for (int c = 0; c < 32; ++c) {
        const float want = (c + 32 * pass == p) ? 1.0f : 0.0f;
        if (o[c] != want) {
          if (bad < 20) printf("p=%d pass=%d col=%d got %g want %g\n", p, pass, c, o[c], want);
          ++bad;
        }
      }
    }
  }
  printf(bad ? "fp4 K pairing: %d MISMATCHES\n" : "fp4 K pairing: A (h,v,n) pairs with B (h,v,n) at all 64 k (%d bad)\n", bad);
  hipFree(d);
  return bad ? 1 : 0;
}
