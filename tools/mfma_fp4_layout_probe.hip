// Maps the operand layout of v_mfma_scale_f32_32x32x64_f8f6f4 with e2m1 (fp4)
// operands on gfx950 with exact 0/1 data.  The packed small-network kernel
// (benor_mfma_small.h) builds a block-diagonal A and needs, for every A
// element (lane, VGPR v, nibble n), its row and the B element (lane, v, n)
// that multiplies the same k.
//   1. rows: A one-hot at (la, v, n), B all ones -> the nonzero output row;
//   2. pairing: A one-hot at (la, v, n), B column c one-hot at position
//      (c + 32 pass, (c >> 3) & 3, c & 7) -> the column that comes out nonzero.
// Prints one line per A lane half and a verdict on the rule
//   row = la & 31, pair = (lane half, v, n) of the B column.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_fp4_layout_probe.hip -o tools/mfma_fp4_layout_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

// out[row * 32 + col]
__global__ void probe(int la, int av, int an, int mode, int pass, float *out) {
  const int lane = threadIdx.x;
  v4i a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
  if (lane == la) a[av] = 0x2 << (4 * an);
  if (mode == 0) {
    b = v4i{0x22222222, 0x22222222, 0x22222222, 0x22222222};
  } else {
    const int c = lane & 31, h = lane >> 5;
    if (h == pass) b[(c >> 3) & 3] = 0x2 << (4 * (c & 7));
  }
  v16f acc = {};
  const v8i a8 = {a[0], a[1], a[2], a[3], 0, 0, 0, 0};
  const v8i b8 = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, acc, 4, 4, 0, 127, 0, 127);
  for (int j = 0; j < 16; ++j) {
    const int row = (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5), col = lane & 31;
    out[row * 32 + col] = acc[j];
  }
}

int main() {
  float *d;
  hipMalloc(&d, 1024 * sizeof(float));
  float o[1024];
  int rule_bad = 0;
  for (int la = 0; la < 64; ++la) {
    for (int av = 0; av < 4; ++av) {
      for (int an = 0; an < 8; ++an) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, la, av, an, 0, 0, d);
        hipMemcpy(o, d, sizeof o, hipMemcpyDeviceToHost);
        int row = -1, nrows = 0;
        for (int r = 0; r < 32; ++r) {
          bool nz = false;
          for (int c = 0; c < 32; ++c) nz |= o[r * 32 + c] != 0.0f;
          if (nz) { row = r; ++nrows; }
        }
        int pair_pass = -1, pair_col = -1, npairs = 0;
        for (int pass = 0; pass < 2; ++pass) {
          hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, la, av, an, 1, pass, d);
          hipMemcpy(o, d, sizeof o, hipMemcpyDeviceToHost);
          for (int r = 0; r < 32; ++r)
            for (int c = 0; c < 32; ++c)
              if (o[r * 32 + c] != 0.0f) { pair_pass = pass; pair_col = c; ++npairs; }
        }
        // B position of the pair: lane half pair_pass, VGPR (col >> 3) & 3, nibble col & 7
        const bool ok = nrows == 1 && row == (la & 31) && npairs == 1 && pair_pass == (la >> 5) &&
                        ((pair_col >> 3) & 3) == av && (pair_col & 7) == an;
        if (!ok) {
          if (rule_bad < 40)
            printf("A lane %2d v%d n%d: row %d (%d rows)  pairs with B half %d v%d n%d (%d pairs)\n", la, av, an, row,
                   nrows, pair_pass, pair_col >= 0 ? (pair_col >> 3) & 3 : -1, pair_col >= 0 ? pair_col & 7 : -1,
                   npairs);
          ++rule_bad;
        }
      }
    }
  }
  printf(rule_bad ? "fp4 layout: %d A elements break the rule\n"
                  : "fp4 layout: row = lane & 31 and A (half, v, n) pairs with B (half, v, n) for all 2048 elements (%d)\n",
         rule_bad);
  hipFree(d);
  return rule_bad ? 1 : 0;
}
