// benor_mfma_big.h -- helpers shared by the big-network matrix-core kernels
// (1024 < m <= 4096): the per-wave form (benor_mfma_big.hip) and the
// workgroup-cooperative form (benor_mfma_coop.hip).
#pragma once

#include "benor_mfma.h"

namespace benor {

constexpr uint32_t kBigMaxW = kMaxW;   // 64 chunks at N = 4096
#ifndef BENOR_BIG_REG_WAVES
// Waves per CU assumed for the workgroup-size choice.  The kernel takes 124-131
// VGPRs (3 waves per SIMD), but choosing as if 2 per SIMD fit measured best
// (12 or 16: -3..-20 % on N=2048..4096 shapes; profiles/r02_big_zero_start_ab.jsonl).
#define BENOR_BIG_REG_WAVES 8
#endif

// Words per lane of a wave's x plane: the W x1 words rounded up to whole
// Philox blocks per lane half (4 words each); the slice adds the KP <= W
// proposal words (+1: a tile block may fill word KP when KP is odd).
__host__ __device__ constexpr uint32_t big_plane_words(uint32_t W) { return 4u * ((((W + 1u) >> 1) + 1u) >> 1); }
// The R-phase writes NT/2 proposal words per block of NT tiles, so up to
// ceil(MT/NT) * NT/2 <= W + NT/2 - 1 words (MT = ceil(m/32) <= 2W).
__host__ __device__ constexpr uint32_t big_prop_words(uint32_t W, uint32_t NT) { return W + NT / 2u - 1u; }
// REGEN (round 1 of random initial values): no x plane in LDS, each tile block
// regenerates its x words from Philox, so the slice is the proposal words only.
__host__ __device__ constexpr uint32_t big_slice_words(uint32_t W, uint32_t NT, bool regen) {
  return (regen ? 0u : big_plane_words(W)) + big_prop_words(W, NT);
}
// Receiver tiles per expanded operand: 8 from W = 28 on (more independent
// accumulator chains and half the expansion VALU and LDS reads per product,
// at 2 waves per SIMD), else 4 (3 waves per SIMD by registers).  Measured
// (profiles/r02_big_nt_ab.jsonl): NT = 8 +20 % at N=4096 F=0 (W=64), +12 % at
// N=2048 F=0 (W=32), +6 % at N=4096 F=2000 (W=33), -2 % at N=4096 F=1365
// (W=43), -8 % at W=21..22.
constexpr uint32_t kBigNt8MinW = 28;
__host__ __device__ constexpr uint32_t big_nt(uint32_t W) { return W >= kBigNt8MinW ? 8u : 4u; }
// The workgroup-cooperative form (benor_mfma_coop.hip) from this W on.
constexpr uint32_t kCoopMinW = 22;

// x1 words of chunks 4j .. 4j+3 of this lane half (h) from /start Philox block
// 2j + h: half h keeps words h and 2 + h of its block and trades the other two
// with lane l ^ 32 (DS bpermute).
__device__ __forceinline__ void big_x_block(const uint32_t *keys, uint64_t trial, uint32_t h, uint32_t j,
                                            uint32_t (&xw)[4]) {
  const uint2 kk = lds_keys(keys);
  const uint4 r = philox4x32_10(kk.x, kk.y, make_uint4((uint32_t)trial, (uint32_t)(trial >> 32), 2u * j + h,
                                                       kStreamInit << 24));
  half_trade(r, h, xw);
}

}  // namespace benor
