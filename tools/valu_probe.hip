// valu_probe.hip -- issue-rate microbenchmark for the VALU ops the round loop
// uses (v_bcnt_u32_b32 popcount+accumulate, v_and_b32, v_add_u32), at full
// occupancy with independent chains.  Prints lane-ops/s and cycles per
// wave64 instruction per SIMD at the clock the part holds.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o tools/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP, int CH = 8>
__global__ void __launch_bounds__(256) probe(unsigned *sink, int iters, unsigned seed) {
  unsigned a[8];
  unsigned long long c[8];
  const unsigned x = threadIdx.x * 2654435761u + blockIdx.x + seed;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = x + (unsigned)i;
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = x ^ (unsigned)i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        if (OP == 0) asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(a[i]) : "v"(x));
        if (OP == 1) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[i]) : "v"(x));
        if (OP == 2) asm volatile("v_and_b32 %0, %1, %0" : "+v"(a[i]) : "v"(x));
        if (OP == 3) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(a[i]) : "v"(x));
        if (OP == 4) asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(a[i]) : "s"(seed));
        if (OP == 5) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "s"(seed + i));
        if (OP == 6) asm volatile("v_writelane_b32 %0, %1, 5" : "+v"(a[i]) : "s"(seed + i));
        if (OP == 7) asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(a[i]), "v"(x) : "vcc");
        if (OP == 8) asm volatile("v_mul_hi_u32 %0, %1, %0" : "+v"(a[i]) : "v"(x));
        if (OP == 9) {
          unsigned long long t;
          asm volatile("v_mov_b64 %0, %1" : "=v"(t) : "s"((unsigned long long)seed << 32 | (unsigned)i));
          a[i] ^= (unsigned)t;
        }
        if (OP == 10) asm volatile("v_not_b32 %0, %0" : "+v"(a[i]));
        if (OP == 11) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[i]) : "s"(seed));
        if (OP == 12) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a[i]) : "v"(x));
        if (OP == 13) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(c[i]) : "v"(x), "v"(a[i]) : "vcc");
        if (OP == 14) asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0x96" : "+v"(a[i]) : "v"(x), "s"(seed));
        if (OP == 15) asm volatile("v_cvt_scalef32_pk_fp4_f32 %0, %1, %1, %2" : "+v"(a[i]) : "v"(x), "v"(1.0f));
        if (OP == 16) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(a[i]) : "v"(x), "s"(0x0C0C0B09u));
        if (OP == 17) asm volatile("v_bfe_u32 %0, %0, 3, 1" : "+v"(a[i]));
        if (OP == 18) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a[i]));
        if (OP == 19) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(x));
        if (OP == 20) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(x));
        if (OP == 21) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(x), "s"((unsigned long long)seed * 0x100000001ull));
        if (OP == 22) asm volatile("v_bfi_b32 %0, %1, %0, %1" : "+v"(a[i]) : "v"(x));
        if (OP == 23) asm volatile("v_bfe_i32 %0, %0, 3, 1" : "+v"(a[i]));
      }
    }
  }
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= a[i] ^ (unsigned)c[i] ^ (unsigned)(c[i] >> 32);
  if (s == 0x12345678u) sink[blockIdx.x] = s;
}

template <int OP, int CH = 8>
void run(const char *name, int cus, int blocks_per_cu, int threads = 256) {
  unsigned *sink;
  (void)hipMalloc(&sink, sizeof(unsigned) * cus * 64);
  const int grid = cus * blocks_per_cu, iters = 4096;
  hipLaunchKernelGGL((probe<OP, CH>), dim3(grid), dim3(threads), 0, 0, sink, iters, 1u);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, 0);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((probe<OP, CH>), dim3(grid), dim3(threads), 0, 0, sink, iters, 1u);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  const double ops = (double)grid * threads * iters * 8 * CH * reps;
  const double rate = ops / (ms * 1e-3);
  if (CH == 8) {
    // cycles per wave64 instruction per SIMD at 2.4 GHz nominal
    const double cyc = (double)cus * 4 * 64 * 2.4e9 / rate;
    printf("%-24s blocks/CU=%2d  %.2f T lane-ops/s  (%.2f cyc/wave-instr/SIMD @2.4GHz)\n", name, blocks_per_cu,
           rate / 1e12, cyc);
  } else {
    // one dependent chain in one wave per CU: cycles from issue to a dependent issue
    const double per_wave = ms * 1e-3 / reps / ((double)iters * 8 * CH);
    printf("%-24s one chain, one wave per CU: %.1f cycles per dependent instruction @2.4GHz\n", name,
           per_wave * 2.4e9);
  }
  (void)hipFree(sink);
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs: %d\n", cus);
  for (int bpc : {8}) {
    run<0>("v_bcnt_u32_b32 (v,v)", cus, bpc);
    run<4>("v_bcnt_u32_b32 (s,v)", cus, bpc);
    run<1>("v_add_u32", cus, bpc);
    run<2>("v_and_b32", cus, bpc);
    run<3>("v_fma_f32", cus, bpc);
    run<5>("v_mov_b32 (s)", cus, bpc);
    run<6>("v_writelane_b32", cus, bpc);
    run<7>("v_cmp_gt_u32", cus, bpc);
    run<8>("v_mul_hi_u32", cus, bpc);
    run<9>("v_mov_b64 (s) + v_xor", cus, bpc);
    run<10>("v_not_b32", cus, bpc);
    run<11>("v_xor_b32 (s,v)", cus, bpc);
    run<12>("v_mul_lo_u32", cus, bpc);
    run<13>("v_mad_u64_u32", cus, bpc);
    run<14>("v_bitop3_b32 (xor3)", cus, bpc);
    run<15>("v_cvt_scalef32_pk_fp4", cus, bpc);
    run<16>("v_perm_b32", cus, bpc);
    run<17>("v_bfe_u32", cus, bpc);
    run<18>("v_lshlrev_b32", cus, bpc);
    run<19>("v_and_or_b32", cus, bpc);
    run<20>("v_cndmask_b32 (vcc)", cus, bpc);
    run<21>("v_cndmask_b32_e64 (s)", cus, bpc);
    run<22>("v_bfi_b32", cus, bpc);
    run<23>("v_bfe_i32", cus, bpc);
  }
  // dependent-issue latency (packed small-network kernel, r03)
  run<1, 1>("v_add_u32", cus, 1, 64);
  run<0, 1>("v_bcnt_u32_b32", cus, 1, 64);
  run<13, 1>("v_mad_u64_u32", cus, 1, 64);
  run<14, 1>("v_bitop3_b32", cus, 1, 64);
  run<15, 1>("v_cvt_scalef32_pk_fp4", cus, 1, 64);
  run<16, 1>("v_perm_b32", cus, 1, 64);
  return 0;
}
