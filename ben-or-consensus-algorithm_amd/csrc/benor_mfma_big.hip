// benor_mfma_big.hip -- the matrix-core round-1 kernel for big networks,
// 1024 < m <= 4096 (W = ceil(m / 64) = 17..64 sender chunks): the same
// formulation, KINDs and deferral as benor_mfma.h, with the chunk count a
// runtime value.
//
// What changes with size.  benor_mfma.h keeps every operand of a trial group
// in registers, fully unrolled per W; at W = 64 that would be 4W VGPRs of
// expanded votes plus 2 * ceil(m/32) of packed proposals.  Here
//  * the x plane stays as bits in the wave's LDS slice, one word per lane
//    per chunk, read and expanded to e2m1 nibbles right before each product
//    (one ds_read_b32 and 4 VALU per two products; runtime loops, so the code
//    does not grow with W and no operand array lives in registers);
//  * the proposal plane goes to LDS as bits too, one word per lane per pair of
//    receiver tiles: the fp4-converted R-phase results (+6 / -6 / 0 nibbles,
//    as KIND 1, 2 of benor_mfma.h) keep their sign bits, four nibble words
//    folding into one 32-bit word (bit 4i + 3 - s of word s), so the P-phase
//    counts c0 = the receivers whose proposal is 0 (node.ts:63-69);
//  * NT receiver tiles run side by side on one expanded operand (NT
//    independent accumulator chains: 1/NT of the expansion VALU and LDS
//    reads per product).
// The layout of accumulators, trial columns and thresholds is benor_mfma.h's;
// the P-phase thresholds are on c0 (A scale 2^0, or 2^1 for KIND 2):
//  KIND 0, 1: acc = c0 - F - 0.5, negative exactly when c0 <= F: with no "?"
//    proposal c1 = m - c0 >= m - F > F, so the receiver decides 1
//    (node.ts:102-105); positive: c0 > F, decide 0 (node.ts:99-101);
//  KIND 2: acc = 2 c0 - m; decided iff |acc| > 2F - m (c0 > F or c1 > F),
//    0 for acc > 0, 1 for acc < 0.
// Trials with a "?" proposal (KIND 1, 2) or an undecided receiver (KIND 2)
// are deferred to the popcount kernel exactly as in benor_mfma.h.
#include "benor_mfma_big.h"

#include <cstdlib>
#include <cstring>

namespace benor {

template <int KIND, int NT, int BW, bool REGEN>
__global__ void __launch_bounds__(64 * BW) benor_mfma_big_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u, h = lane >> 5;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  // Continuation pass (KIND > 0): round `cont` of the listed trials, from the
  // coins of round cont-1 (benor_mfma.h).
  const uint32_t cont = KIND == 0 ? 0u : p.cont_round;
  uint32_t m = p.m, W = p.W, hist_len = p.hist_len;
  uint32_t trial_count = cont ? *p.trial_list_len : (uint32_t)p.trial_count;
  asm volatile("" : "+s"(m), "+s"(W), "+s"(hist_len), "+s"(trial_count));
  const uint32_t MT = (m + 31u) >> 5;         // 32-receiver tiles
  const uint32_t KP = (MT + 1u) >> 1;         // P-phase K chunks (tile pairs)

  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint32_t *keys = reinterpret_cast<uint32_t *>(smem + p.hist_bytes - kParamBytes);
  // The wave's LDS slice: X [plane_words][64] x1 bits, then P [W][64]
  // proposal bits.  Each lane reads back only its own words (its trial
  // column and half), so no barrier orders them.
  uint32_t *X = reinterpret_cast<uint32_t *>(smem + p.hist_bytes) + (size_t)wv * big_slice_words(W, NT, REGEN) * 64u;
  uint32_t *PL = X + (REGEN ? 0u : big_plane_words(W)) * 64u;
  for (uint32_t i = threadIdx.x; i < hist_len; i += blockDim.x) lhist[i] = 0u;
  if (threadIdx.x == 0) {
    keys[0] = (uint32_t)p.seed;
    keys[1] = (uint32_t)(p.seed >> 32);
    keys[2] = (uint32_t)p.trial_begin;
    keys[3] = (uint32_t)(p.trial_begin >> 32);
  }
  __syncthreads();

  const bool random_init = p.init_mode == BO_INIT_RANDOM;
  const float bias_r = -8.0f * (float)(cont ? m : m - p.init_q);   // acc = 8 (c1 - c0): p1 > 0, p0 < 0, "?" = 0
  const float bias_p = KIND == 2 ? -(float)m : -((float)p.F + 0.5f);
  const float dec_thr = (float)(2u * p.F - m) + 0.5f;   // KIND 2: |2 c0 - m| > 2F - m <=> decided
  const uint32_t mrem = m - 32u * (MT - 1u);             // live rows of the last tile, 1..32
  uint32_t tail0 = 0, tail1 = 0;                         // its nibble masks (KIND-1-style packing)
  uint32_t live_last = 0;                                // its live accumulator registers
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t row = (uint32_t)((j & 3) + 8 * (j >> 2)) + 4u * h;
    if (row < mrem) {
      live_last |= 1u << j;
      if (j < 8) tail0 |= 0xFu << (4 * (j & 7));
      else tail1 |= 0xFu << (4 * (j & 7));
    }
  }
  const int last_bits = (int)m - 32 * (2 * ((int)W - 1) + (int)h);
  const uint32_t last_mask = last_bits >= 32 ? ~0u : (last_bits <= 0 ? 0u : ((1u << last_bits) - 1u));

  mf_v4i ones = {0x22222222, 0x22222222, 0x22222222, 0x22222222};
  uint32_t f_all = 0, f_1 = 0, f_2 = 0;
  const uint32_t ngroups = (trial_count + 31u) >> 5;
  const uint32_t waves_total = gridDim.x * BW;
  const uint32_t wave_id = blockIdx.x * BW + wv;
  uint32_t n_def = 0;
  uint32_t *seg = KIND == 0 ? nullptr : p.defer_seg + (size_t)wave_id * p.defer_seg_cap;
  for (uint32_t g = wave_id; g < ngroups; g += waves_total) {
    const uint32_t t = (g << 5) + (lane & 31u);
    const bool valid = t < trial_count;
    const uint32_t toff = cont ? (valid ? p.trial_list[t] : 0u) : t;   // the trial's offset in the launch
    // ---- /start (node.ts:167-188): x1 words 2c + h of this lane's trial, c < W
    if (REGEN) {
      // x words are regenerated per tile block in the R-phase
    } else if (KIND != 0 && cont != 0u) {      // continuation: the coins of round cont-1
      const uint64_t trial = lds_u64(keys + 2) + toff;
      for (uint32_t c = 0; c < W; ++c) {
        const uint2 kk = lds_keys(keys);
        const uint4 r = coin_block(kk.x, kk.y, (uint32_t)trial, (uint32_t)(trial >> 32), 32u * (2u * c + h), cont - 1u);
        X[c * 64u + lane] = coin_word(r, cont - 1u);
      }
    } else if (random_init) {                  // whole Philox blocks, the halves trading words
      const uint64_t trial = lds_u64(keys + 2) + t;
      const uint32_t NJ = (((W + 1u) >> 1) + 1u) >> 1;   // blocks per lane half
      for (uint32_t j = 0; j < NJ; ++j) {
        const uint2 kk = lds_keys(keys);
        const uint4 r = philox4x32_10(kk.x, kk.y,
                                      make_uint4((uint32_t)trial, (uint32_t)(trial >> 32), 2u * j + h, kStreamInit << 24));
        uint32_t q4[4];
        half_trade(r, h, q4);
        for (uint32_t q = 0; q < 4u; ++q) X[(4u * j + q) * 64u + lane] = q4[q];
      }
    } else {
      for (uint32_t c = 0; c < W; ++c) {
        const uint4 q = p.init_plane[c];
        X[c * 64u + lane] = h ? q.w : q.z;
      }
    }
    if (!REGEN) X[(W - 1u) * 64u + lane] &= last_mask;

    // ---- R-phase (node.ts:46-82): NT receiver tiles on each expanded x
    // chunk; proposals to LDS as sign bits (1 = proposal 0).
    uint32_t qz = 0u;
    for (uint32_t i = 0; i < MT; i += (uint32_t)NT) {
      // Accumulators start at 0 and take their bias after the chunk loop: a
      // bias-splat start value kept a second 16-register tuple per tile live
      // across the loop (occupancy 2 -> 3-4 waves per SIMD without it).
      mf_v16f acc[NT];
#pragma unroll
      for (int u = 0; u < NT; ++u) acc[u] = mf_v16f{};
      if constexpr (REGEN) {
        // x1 words of chunks 4j .. 4j+3 from Philox block 2j + h, the lane
        // halves trading two words (as the /start code of the LDS form).
        // Blocks before the last hold 4 full chunks (none is chunk W - 1):
        // block j + 1's Philox is issued among block j's 4 NT products, one
        // MFMA and a few VALU at a time, so it runs in the products' shadow.
        const uint64_t trial = lds_u64(keys + 2) + t;
        const uint32_t NJ = (((W + 1u) >> 1) + 1u) >> 1;
        uint32_t xw[4];
        big_x_block(keys, trial, h, 0u, xw);
        for (uint32_t j = 0; j + 1u < NJ; ++j) {
          uint32_t xn[4];
          big_x_block(keys, trial, h, j + 1u, xn);
#pragma unroll
          for (uint32_t q = 0; q < 4u; ++q) {
            const mf_v4i b = expand_votes(xw[q]);
#pragma unroll
            for (int u = 0; u < NT; ++u) {
              asm volatile("" : "+v"(ones));
              acc[u] = mfma_count<4>(ones, b, acc[u]);
            }
          }
#pragma unroll
          for (int k = 0; k < 4 * NT; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);   // up to three VALU
          }
#pragma unroll
          for (uint32_t q = 0; q < 4u; ++q) xw[q] = xn[q];
        }
        // the last block: chunks 4 (NJ - 1) .. W - 1, chunk W - 1 masked
#pragma unroll
        for (uint32_t q = 0; q < 4u; ++q) {
          const uint32_t c = 4u * (NJ - 1u) + q;
          if (c < W) {
            const mf_v4i b = expand_votes(c == W - 1u ? xw[q] & last_mask : xw[q]);
#pragma unroll
            for (int u = 0; u < NT; ++u) {
              asm volatile("" : "+v"(ones));
              acc[u] = mfma_count<4>(ones, b, acc[u]);
            }
          }
        }
      } else {
        // chunk c + 1's x word is read from LDS among chunk c's NT products
        uint32_t wcur = X[lane];
        for (uint32_t c = 0; c < W; ++c) {
          const uint32_t wnext = X[(c + 1u < W ? c + 1u : c) * 64u + lane];
          const mf_v4i b = expand_votes(wcur);
#pragma unroll
          for (int u = 0; u < NT; ++u) {
            asm volatile("" : "+v"(ones));     // opaque per tile: no two tiles' products merge
            acc[u] = mfma_count<4>(ones, b, acc[u]);
          }
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);     // the next word's read first
#pragma unroll
          for (int k = 0; k < NT; ++k) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          wcur = wnext;
        }
      }
#pragma unroll
      for (int u = 0; u < NT; ++u)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[u][j] += bias_r;
#pragma unroll
      for (int q = 0; q < NT / 2; ++q) {      // tile pair (i + 2q, i + 2q + 1) -> proposal word (i >> 1) + q
        uint32_t n[4];
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const uint32_t ti = i + 2u * q + v;  // nibble masks: full, the last (partial) tile, or none (past MT)
          const uint32_t k0 = ti < MT - 1u ? ~0u : (ti == MT - 1u ? tail0 : 0u);
          const uint32_t k1 = ti < MT - 1u ? ~0u : (ti == MT - 1u ? tail1 : 0u);
          n[2 * v] = pack_fp4_8(acc[2 * q + v], 0) & k0;
          n[2 * v + 1] = pack_fp4_8(acc[2 * q + v], 8) & k1;
          if constexpr (KIND > 0)              // a live "?" nibble is 0: bit 1 clear
            qz |= (~n[2 * v] & k0 & 0x22222222u) | (~n[2 * v + 1] & k1 & 0x22222222u);
        }
        const uint32_t s = 0x88888888u;
        PL[((i >> 1) + q) * 64u + lane] = (n[0] & s) | ((n[1] & s) >> 1) | ((n[2] & s) >> 2) | ((n[3] & s) >> 3);
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- P-phase (node.ts:83-158): every receiver tile counts the 0-proposals
    float mn = __builtin_inff(), mx = -__builtin_inff(), ma = __builtin_inff();
    for (uint32_t i = 0; i < MT; i += (uint32_t)NT) {
      const float nanf = __builtin_nanf("");
      mf_v16f acc[NT];
#pragma unroll
      for (int u = 0; u < NT; ++u) acc[u] = mf_v16f{};
      uint32_t wcur = PL[lane];                // chunk k + 1's word read among chunk k's products
      for (uint32_t k = 0; k < KP; ++k) {
        const uint32_t wnext = PL[(k + 1u < KP ? k + 1u : k) * 64u + lane];
        const mf_v4i b = expand_votes(wcur);
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          asm volatile("" : "+v"(ones));
          acc[u] = KIND == 2 ? mfma_count<1>(ones, b, acc[u]) : mfma_count(ones, b, acc[u]);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
        for (int u = 0; u < NT; ++u) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        wcur = wnext;
      }
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const uint32_t ti = i + u;
        if (ti + 1u < MT) {
#pragma unroll
          for (int j = 0; j < 16; ++j) acc[u][j] += bias_p;
        } else {                               // rows with no receiver become NaN: the reductions skip them
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const bool live = ti == MT - 1u && ((live_last >> j) & 1u);
            acc[u][j] += live ? bias_p : nanf;
          }
        }
#pragma unroll
        for (int j = 0; j < 16; j += 2) {
          mn = fminf(fminf(mn, acc[u][j]), acc[u][j + 1]);
          mx = fmaxf(fmaxf(mx, acc[u][j]), acc[u][j + 1]);
          if constexpr (KIND == 2) ma = fminf(fminf(ma, __builtin_fabsf(acc[u][j])), __builtin_fabsf(acc[u][j + 1]));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- outcome: bins 3R + v; KIND > 0 defers as benor_mfma.h
    uint32_t halt = (uint32_t)ballot(valid);
    if constexpr (KIND > 0) {
      const bool defer = qz != 0u || (KIND == 2 && !(ma > dec_thr));
      const uint64_t bd = ballot(valid && defer);
      const uint32_t dcols = (uint32_t)bd | (uint32_t)(bd >> 32);
      halt &= ~dcols;
      if (dcols) {
        if (lane < 32u && ((dcols >> lane) & 1u)) {
          // the host sizes a segment for a wave's most groups per launch
          // (plan_launch_impl); the bound only guards the buffer
          const uint32_t idx = n_def + (uint32_t)__builtin_popcount(dcols & ((1u << lane) - 1u));
          if (idx < p.defer_seg_cap) seg[idx] = toff;   // beyond: counted, flagged below
        }
        n_def += (uint32_t)__builtin_popcount(dcols);
      }
    }
    // KIND 0, 1: acc < 0 <=> decided 1; KIND 2: acc < 0 <=> decided 1 as well (2 c0 - m < 0)
    const uint64_t b1 = ballot(mn < 0.0f);
    const uint64_t b0 = ballot(mx > 0.0f);
    const uint32_t any1 = ((uint32_t)b1 | (uint32_t)(b1 >> 32)) & halt;
    const uint32_t any0 = ((uint32_t)b0 | (uint32_t)(b0 >> 32)) & halt;
    f_all += (uint32_t)__builtin_popcount(halt);
    f_1 += (uint32_t)__builtin_popcount(any1);
    f_2 += (uint32_t)__builtin_popcount(any1 & any0);
  }
  if constexpr (KIND > 0) {
    // the waves' deferred trials -> the compact list, one global atomic per
    // workgroup (as benor_mfma.h; parameter-block words 4..7, BW <= 4)
    if (n_def > p.defer_seg_cap) {   // segment overflow: the extra trials are dropped and the launch flagged
      if (lane == 0) atomicOr(p.overflow, 1u);
      n_def = p.defer_seg_cap;
    }
    uint32_t *wdef = keys + 4;
    if (lane == 0) wdef[wv] = n_def;
    __syncthreads();
    uint32_t before = 0u, total = 0u;
#pragma unroll
    for (uint32_t w = 0; w < (uint32_t)BW; ++w) {
      const uint32_t c = wdef[w];
      total += c;
      before += w < wv ? c : 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0 && total) wdef[0] = atomicAdd(p.defer_len, total);
    __syncthreads();
    if (n_def) {
      const uint32_t base = wdef[0] + before;
      for (uint32_t i = lane; i < n_def; i += 64u) p.defer_list[base + i] = seg[i];
    }
  }

  const uint32_t rb = 3u * (cont ? cont : 1u);   // bins 3R + v of the halting round R
  const uint32_t hc = lane == rb ? f_all - f_1 : (lane == rb + 1u ? f_1 - f_2 : (lane == rb + 2u ? f_2 : 0u));
  if (hc) atomicAdd(&lhist[lane], hc);
  if (lane == 0 && f_2) atomicAdd(&lhist[hist_len - 1u], f_2);
  __syncthreads();
  flush_hist(lhist, p);
}

// Round 1 of random initial values regenerates its x words from Philox (no x
// plane in LDS) when the LDS form's slices would hold the CU under 2 waves per
// SIMD (from W ~ 39): +12 % at N=4096 F=1365 (W=43, 6 -> 8 waves per CU), +8 %
// at N=4096 F=0 (W=64, 4 -> 8); where the LDS form already fits 8 waves the
// extra Philox VALU costs 4-10 % (profiles/r02_big_regen_ab.jsonl).
static bool big_regen(const KParams &p) {
  if (p.init_mode != BO_INIT_RANDOM || p.cont_round != 0u) return false;
  return lds_groups_per_cu(p.hist_bytes + big_slice_words(p.W, big_nt(p.W), false) * 64u * 4u) < 8u;
}

uint32_t mfma_big_lds_bytes(const KParams &p, uint32_t bw) {
  return p.hist_bytes + bw * big_slice_words(p.W, big_nt(p.W), big_regen(p)) * 64u * 4u;
}

// Waves per workgroup: the most resident waves per CU -- LDS (160 KB) against
// the ~2 waves/SIMD its registers allow -- with ties to larger workgroups,
// which spread over the CU's four SIMDs.  (Measured at NT = 4: 1-wave groups
// +22 % at N=4096, F=1365, where LDS admits 7 single waves but one 4-wave
// group; -10..-30 % where both fill the CU.)
uint32_t mfma_big_block_waves(const KParams &p) {
  constexpr uint32_t kRegWaves = BENOR_BIG_REG_WAVES;
  uint32_t best = 4, best_waves = 0;
  for (uint32_t bw = 4; bw >= 1; bw >>= 1) {
    uint32_t w = lds_groups_per_cu(mfma_big_lds_bytes(p, bw)) * bw;
    if (w > kRegWaves) w = kRegWaves;
    if (w > best_waves) {
      best_waves = w;
      best = bw;
    }
  }
  return best;
}

template <int KIND, int NT, int BW, bool REGEN>
static hipError_t launch_big_regen(const KParams &p, int grid, hipStream_t s) {
  const uint32_t lds = mfma_big_lds_bytes(p, BW);
  if (lds > 64u * 1024u) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&benor_mfma_big_kernel<KIND, NT, BW, REGEN>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((benor_mfma_big_kernel<KIND, NT, BW, REGEN>), dim3(grid), dim3(64 * BW), lds, s, p);
  return hipGetLastError();
}

template <int KIND, int NT, int BW>
static hipError_t launch_big_kind(const KParams &p, int grid, hipStream_t s) {
  return big_regen(p) ? launch_big_regen<KIND, NT, BW, true>(p, grid, s) : launch_big_regen<KIND, NT, BW, false>(p, grid, s);
}

template <int KIND, int NT>
static hipError_t launch_big_bw(const KParams &p, int grid, hipStream_t s) {
  const uint32_t bw = mfma_big_block_waves(p);
  if (bw == 4u) return launch_big_kind<KIND, NT, 4>(p, grid, s);
  if (bw == 2u) return launch_big_kind<KIND, NT, 2>(p, grid, s);
  return launch_big_kind<KIND, NT, 1>(p, grid, s);
}

template <int KIND>
static hipError_t launch_big_nt(const KParams &p, int grid, hipStream_t s) {
  return big_nt(p.W) == 8u ? launch_big_bw<KIND, 8>(p, grid, s) : launch_big_bw<KIND, 4>(p, grid, s);
}

// The cooperative form (benor_mfma_coop.hip) from W = 22 on; below, the
// per-wave form.  Measured (r03-s2b, profiles/r03-s2b_coop_ab.txt, node-rounds
// per second, coop vs per-wave): N=4096 F=0 at 10^5 trials x1.69 (the
// per-wave form's long group tail), 10^6 x1.17; N=4096 F=1365 (W=43) x1.06-1.10;
// N=3000 F=1400 (W=25) x1.06; N=2048 F=682 (W=22) x1.09; N=1500 F=200 (W=21)
// x1.01; N=2049 F=1024 (W=17, KIND 2) x0.93.  BENOR_BIG_FORM=wave / coop
// forces one (validation knob: tests run both forms at every W).
bool mfma_big_coop(const KParams &p) {
  if (p.variant != 7 || p.W <= 16u || p.node_out || p.rounds_out) return false;
  if (knob_is("BENOR_BIG_FORM", "wave")) return false;
  if (knob_is("BENOR_BIG_FORM", "coop")) return true;
  return p.W >= kCoopMinW;
}

hipError_t launch_mfma_big(const KParams &p, int grid, hipStream_t s) {
  if (p.W < 17u || p.W > kBigMaxW) return hipErrorInvalidValue;
  if (mfma_big_coop(p)) return launch_mfma_coop(p, grid, s);
  if (p.G == 0u) return launch_big_nt<0>(p, grid, s);
  if (p.G == 1u) return launch_big_nt<1>(p, grid, s);
  return launch_big_nt<2>(p, grid, s);
}

}  // namespace benor
