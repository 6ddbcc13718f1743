// Phase timing of the packed small-network kernel (benor_mfma_small.h built
// with BENOR_SMALL_TIMING): shader-clock cycles per wave iteration spent in
// refill, Philox, R-phase, P-phase, slot updates.  Random initial values,
// first F nodes faulty.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DBENOR_SMALL_TIMING -I include \
//     -I ben-or-consensus-algorithm_amd/csrc -mllvm -amdgpu-mfma-vgpr-form \
//     tools/small_phase_probe.hip -o tools/small_phase_probe
//   tools/small_phase_probe [trials] [blocks_per_cu]
#include <stdio.h>
#include <stdlib.h>

#include "benor_mfma_small.h"

using namespace benor;

int main(int argc, char **argv) {
  const uint64_t T = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1000000ull;
  const int bpc = argc > 2 ? atoi(argv[2]) : 1;
  constexpr int MM = 6;
  KParams p{};
  p.N = 10;
  p.F = 4;
  p.m = MM;
  p.W = 1;
  p.k_max = 16;
  p.init_mode = BO_INIT_RANDOM;
  p.seed = 0x243F6A8885A308D3ull;
  p.trial_begin = 0;
  p.trial_count = T;
  p.hist_len = (p.k_max + 1u) * 3u + 1u;
  p.hist_bytes = (((p.hist_len * 4u) + 15u) & ~15u) + kParamBytes;
  p.lds_bytes = p.hist_bytes;
  unsigned long long *hist, *tim;
  hipMalloc(&hist, 8 * p.hist_len);
  const size_t tim_words = 8 + 3 * 256 * 16 * 4;
  hipMalloc(&tim, 8 * tim_words);
  hipMemset(hist, 0, 8 * p.hist_len);
  hipMemset(tim, 0, 8 * tim_words);
  p.hist = hist;
  p.rounds_out = reinterpret_cast<uint32_t *>(tim);
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const uint64_t groups = (T + 64 * small_slots(MM) - 1) / (64 * small_slots(MM));
  uint64_t grid = (uint64_t)cus * bpc, need = (groups + 3) / 4;
  if (need < grid) grid = need;
  launch_mfma_small_m<MM>(p, (int)grid, 0);    // warm-up
  hipDeviceSynchronize();
  hipMemset(tim, 0, 8 * tim_words);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, 0);
  launch_mfma_small_m<MM>(p, (int)grid, 0);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  static unsigned long long t[8 + 3 * 256 * 16 * 4];
  hipMemcpy(t, tim, 8 * tim_words, hipMemcpyDeviceToHost);
  const double it = (double)t[6] / (double)t[7];
  printf("trials %llu grid %llu blocks, %.1f us; waves %llu, %.2f iterations per wave\n", (unsigned long long)T,
         (unsigned long long)grid, ms * 1e3, t[7], it);
  const char *names[5] = {"refill/loop", "philox", "x -> R-phase", "P-phase", "slots"};
  double tot = 0;
  for (int i = 0; i < 5; ++i) tot += (double)t[i];
  for (int i = 0; i < 5; ++i)
    printf("  %-14s %8.0f cycles per wave iteration (%4.1f %%)\n", names[i], (double)t[i] / (double)t[6],
           100.0 * (double)t[i] / tot);
  printf("  total          %8.0f cycles per wave iteration\n", tot / (double)t[6]);
  // per wave spans: kernel clock rate, imbalance
  const uint64_t nw = t[7];
  unsigned long long t0 = ~0ull, t1 = 0, itmax = 0;
  double span_sum = 0, span_max = 0, late_start = 0;
  for (uint64_t w = 0; w < nw; ++w) {
    const unsigned long long *r = &t[8 + 3 * w];
    if (r[0] < t0) t0 = r[0];
    if (r[1] > t1) t1 = r[1];
    if (r[2] > itmax) itmax = r[2];
  }
  for (uint64_t w = 0; w < nw; ++w) {
    const unsigned long long *r = &t[8 + 3 * w];
    const double sp = (double)(r[1] - r[0]);
    span_sum += sp;
    if (sp > span_max) span_max = sp;
    if ((double)(r[0] - t0) > late_start) late_start = (double)(r[0] - t0);
  }
  printf("  kernel span %.0f cycles (%.2f GHz vs event time), wave span avg %.0f max %.0f, latest start %.0f, "
         "iterations max %llu\n", (double)(t1 - t0), (double)(t1 - t0) / (ms * 1e6), span_sum / nw, span_max, late_start,
         itmax);
  return 0;
}
