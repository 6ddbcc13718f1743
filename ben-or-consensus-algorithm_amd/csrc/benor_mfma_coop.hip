// benor_mfma_coop.hip -- the big-network matrix-core kernel (1024 < m <= 4096)
// in workgroup-cooperative form: the BW waves of a workgroup run ONE 32-trial
// group together, each wave a share of its receiver tiles.
//
// The per-wave form (benor_mfma_big.hip) gives a whole group to one wave: at
// W = 64 that is 2 * 128 * 64 = 16384 products per group, ~220 us for one
// wave alone on its SIMD.  So a launch whose groups do not fill every wave
// slot many times over ends in a long tail: 10^5 trials at N = 4096 are 3125
// groups on 2048 slots (two rounds of slots, the second half empty), and a
// continuation pass over the ~1.2 % of trials that tied (40 groups) keeps
// 40 SIMDs busy for the full group time.  Here a group takes 1/BW of that,
// and the launch is quantised in groups of BW waves' work.
//
// Layout.  The workgroup's LDS holds ONE x plane (x1 bits, [chunk][lane])
// and ONE proposal plane (sign bits, [tile pair][lane]) instead of one slice
// per wave, so the x plane stays in LDS at every W (no Philox regeneration per
// tile block, benor_mfma_big.hip's REGEN) and more workgroups fit a CU.  One
// group, three barriers:
//   1. /start: the waves write the x words (Philox blocks, coin words or the
//      fixed plane) of the chunks they own (c = wv, wv + BW, ...);
//   2. R-phase (node.ts:46-82): wave wv runs tile blocks wv, wv + BW, ... (NT
//      tiles each, NT accumulator chains on each expanded x word, exactly the
//      per-wave form's block) and writes their proposal words;
//   3. P-phase (node.ts:83-158): the same tile blocks count the proposal
//      plane; each wave's outcome columns (some receiver decided 1 / 0, a
//      column to defer) go to LDS as three 32-bit column masks, and wave 0
//      ORs them and records the group (histogram counters, deferral segment).
// Thresholds, packing, padding and KINDs are the per-wave form's
// (benor_mfma_big.hip header); the outcome of a group is the OR over its
// receivers whichever wave counted them, so histograms are identical.
// Deferred trials go to one segment per workgroup (KParams::defer_seg,
// blockIdx.x * defer_seg_cap), appended to the compact list by wave 0.
#include "benor_mfma_big.h"

#include <type_traits>

namespace benor {

// The x and proposal words as product operands: EXP planes hold them expanded
// (the four e2m1 dwords of expand_votes), so a block's chunk costs one
// ds_read_b128 instead of a ds_read_b32 and the expansion, which every one of
// the MT / NT tile blocks would repeat.
__device__ __forceinline__ mf_v4i as_votes(uint32_t w) { return expand_votes(w); }
__device__ __forceinline__ mf_v4i as_votes(mf_v4i v) { return v; }

// Each tile's first product takes the phase's bias as its C operand (no
// accumulator zeroing, no bias add per result) -- in the P-phase for blocks
// without the last tile, whose dead rows need NaN (r03: +2-4 % against zeroed
// accumulators; profiles/r03-s3k_coop_exp_inproc.jsonl).
// The next group's /start words are written right after this group's P-phase
// products (X is free once the R-phase barrier has passed), so the P-phase
// barrier also publishes them and a group needs two barriers, not three.
template <int KIND, int NT, int BW, bool EXP>
__global__ void __launch_bounds__(64 * BW) benor_mfma_coop_kernel(KParams p) {
  using XW = std::conditional_t<EXP, mf_v4i, uint32_t>;
  constexpr uint32_t XS = EXP ? 4u : 1u;      // dwords per plane word
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u, h = lane >> 5;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t cont = KIND == 0 ? 0u : p.cont_round;
  uint32_t m = p.m, W = p.W, hist_len = p.hist_len;
  uint32_t trial_count = cont ? *p.trial_list_len : (uint32_t)p.trial_count;
  asm volatile("" : "+s"(m), "+s"(W), "+s"(hist_len), "+s"(trial_count));
  const uint32_t MT = (m + 31u) >> 5;         // 32-receiver tiles
  const uint32_t KP = (MT + 1u) >> 1;         // P-phase K chunks (tile pairs)
  const uint32_t NB = (MT + (uint32_t)NT - 1u) / (uint32_t)NT;   // tile blocks

  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint32_t *keys = reinterpret_cast<uint32_t *>(smem + p.hist_bytes - kParamBytes);
  uint32_t *X = reinterpret_cast<uint32_t *>(smem + p.hist_bytes);   // [big_plane_words(W)][64]
  uint32_t *PL = X + big_plane_words(W) * 64u * XS;                   // [big_prop_words(W, NT)][64]
  uint32_t *RED = PL + big_prop_words(W, NT) * 64u * XS;              // [BW][4] column masks
  XW *const XR = reinterpret_cast<XW *>(X);
  XW *const PR = reinterpret_cast<XW *>(PL);
  auto put = [&](XW *plane, uint32_t c, uint32_t w) {   // word c of this lane
    if constexpr (EXP) plane[c * 64u + lane] = expand_votes(w);
    else plane[c * 64u + lane] = w;
  };
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
  uint32_t tail0 = 0, tail1 = 0, live_last = 0;
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
  mf_v16f cb_r, cb_p;
#pragma unroll
  for (int j = 0; j < 16; ++j) cb_r[j] = bias_r, cb_p[j] = bias_p;
  uint32_t f_all = 0, f_1 = 0, f_2 = 0;        // wave 0's counters
  const uint32_t ngroups = (trial_count + 31u) >> 5;
  uint32_t n_def = 0;
  uint32_t *seg = KIND == 0 ? nullptr : p.defer_seg + (size_t)blockIdx.x * p.defer_seg_cap;
  // ---- /start (node.ts:167-188): x1 words 2c + h of group g's trials, the
  // chunks split over the waves
  auto start_x = [&](uint32_t g) {
    const uint32_t t = (g << 5) + (lane & 31u);
    const uint32_t toff = cont ? (t < trial_count ? p.trial_list[t] : 0u) : t;
    if (KIND != 0 && cont != 0u) {             // continuation: the coins of round cont-1
      const uint64_t trial = lds_u64(keys + 2) + toff;
      for (uint32_t c = wv; c < W; c += BW) {
        const uint2 kk = lds_keys(keys);
        const uint4 r = coin_block(kk.x, kk.y, (uint32_t)trial, (uint32_t)(trial >> 32), 32u * (2u * c + h), cont - 1u);
        const uint32_t w = coin_word(r, cont - 1u);
        put(XR, c, c == W - 1u ? w & last_mask : w);
      }
    } else if (random_init) {                  // whole Philox blocks, the halves trading words
      const uint64_t trial = lds_u64(keys + 2) + t;
      const uint32_t NJ = (((W + 1u) >> 1) + 1u) >> 1;   // blocks per lane half
      for (uint32_t j = wv; j < NJ; j += BW) {
        uint32_t xw[4];
        big_x_block(keys, trial, h, j, xw);
#pragma unroll
        for (uint32_t q = 0; q < 4u; ++q) {
          const uint32_t c = 4u * j + q;
          put(XR, c, c == W - 1u ? xw[q] & last_mask : xw[q]);
        }
      }
    } else {
      for (uint32_t c = wv; c < W; c += BW) {
        const uint4 q = p.init_plane[c];
        const uint32_t w = h ? q.w : q.z;
        put(XR, c, c == W - 1u ? w & last_mask : w);
      }
    }
  };
  if (blockIdx.x < ngroups) start_x(blockIdx.x);
  __syncthreads();
  for (uint32_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const uint32_t t = (g << 5) + (lane & 31u);
    const bool valid = t < trial_count;
    const uint32_t toff = cont ? (valid ? p.trial_list[t] : 0u) : t;   // the trial's offset in the launch

    // ---- R-phase: this wave's tile blocks; proposals to LDS as sign bits
    // (1 = proposal 0), packed as in benor_mfma_big.hip
    uint32_t qz = 0u;
    for (uint32_t b = wv; b < NB; b += BW) {
      const uint32_t i = b * (uint32_t)NT;
      mf_v16f acc[NT];
      XW wcur = XR[lane];                      // chunk c + 1's word read among chunk c's products
      {                                        // chunk 0 with C = the bias (W >= 17)
        const XW wnext = XR[64u + lane];
        const mf_v4i bx = as_votes(wcur);
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          asm volatile("" : "+v"(ones));
          acc[u] = mfma_count<4>(ones, bx, cb_r);
        }
        wcur = wnext;
      }
      for (uint32_t c = 1; c < W; ++c) {
        const XW wnext = XR[(c + 1u < W ? c + 1u : c) * 64u + lane];
        const mf_v4i bx = as_votes(wcur);
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          asm volatile("" : "+v"(ones));       // opaque per tile: no two tiles' products merge
          acc[u] = mfma_count<4>(ones, bx, acc[u]);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
        for (int k = 0; k < NT; ++k) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        wcur = wnext;
      }
#pragma unroll
      for (int q = 0; q < NT / 2; ++q) {      // tile pair (i + 2q, i + 2q + 1) -> proposal word (i >> 1) + q
        uint32_t n[4];
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const uint32_t ti = i + 2u * q + v;
          const uint32_t k0 = ti < MT - 1u ? ~0u : (ti == MT - 1u ? tail0 : 0u);
          const uint32_t k1 = ti < MT - 1u ? ~0u : (ti == MT - 1u ? tail1 : 0u);
          n[2 * v] = pack_fp4_8(acc[2 * q + v], 0) & k0;
          n[2 * v + 1] = pack_fp4_8(acc[2 * q + v], 8) & k1;
          if constexpr (KIND > 0)              // a live "?" nibble is 0: bit 1 clear
            qz |= (~n[2 * v] & k0 & 0x22222222u) | (~n[2 * v + 1] & k1 & 0x22222222u);
        }
        const uint32_t s = 0x88888888u;
        put(PR, (i >> 1) + q, (n[0] & s) | ((n[1] & s) >> 1) | ((n[2] & s) >> 2) | ((n[3] & s) >> 3));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();

    // ---- P-phase: this wave's tile blocks count the 0-proposals
    float mn = __builtin_inff(), mx = -__builtin_inff(), ma = __builtin_inff();
    for (uint32_t b = wv; b < NB; b += BW) {
      const uint32_t i = b * (uint32_t)NT;
      const float nanf = __builtin_nanf("");
      const bool cbb = i + (uint32_t)NT < MT;   // every tile of the block has 32 live rows
      mf_v16f acc[NT];
      XW wcur = PR[lane];
      uint32_t k0 = 0;
      if (cbb) {                               // chunk 0 with C = the bias (KP >= 17)
        const XW wnext = PR[64u + lane];
        const mf_v4i bp = as_votes(wcur);
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          asm volatile("" : "+v"(ones));
          acc[u] = KIND == 2 ? mfma_count<1>(ones, bp, cb_p) : mfma_count(ones, bp, cb_p);
        }
        wcur = wnext;
        k0 = 1;
      } else {
#pragma unroll
        for (int u = 0; u < NT; ++u) acc[u] = mf_v16f{};
      }
      for (uint32_t k = k0; k < KP; ++k) {
        const XW wnext = PR[(k + 1u < KP ? k + 1u : k) * 64u + lane];
        const mf_v4i bp = as_votes(wcur);
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          asm volatile("" : "+v"(ones));
          acc[u] = KIND == 2 ? mfma_count<1>(ones, bp, acc[u]) : mfma_count(ones, bp, acc[u]);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
        for (int u = 0; u < NT; ++u) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        wcur = wnext;
      }
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const uint32_t ti = i + u;
        if (cbb) {
        } else if (ti + 1u < MT) {
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
    if (g + gridDim.x < ngroups) start_x(g + gridDim.x);
    // this wave's columns: some receiver decided 1 / 0 (KIND 0, 1, 2: acc < 0
    // <=> decided 1), a "?" proposal or an undecided receiver (defer)
    {
      const bool defer = KIND > 0 && (qz != 0u || (KIND == 2 && !(ma > dec_thr)));
      const uint64_t b1 = ballot(mn < 0.0f), b0 = ballot(mx > 0.0f), bd = ballot(defer);
      if (lane == 0) {
        RED[4u * wv + 0u] = (uint32_t)b1 | (uint32_t)(b1 >> 32);
        RED[4u * wv + 1u] = (uint32_t)b0 | (uint32_t)(b0 >> 32);
        RED[4u * wv + 2u] = (uint32_t)bd | (uint32_t)(bd >> 32);
      }
    }
    __syncthreads();
    // ---- outcome (wave 0): bins 3R + v; KIND > 0 defers as benor_mfma.h
    if (wv == 0u) {
      uint32_t any1 = 0u, any0 = 0u, dcols = 0u;
#pragma unroll
      for (int w = 0; w < BW; ++w) {
        any1 |= RED[4 * w + 0];
        any0 |= RED[4 * w + 1];
        dcols |= RED[4 * w + 2];
      }
      uint32_t halt = (uint32_t)ballot(valid);
      if constexpr (KIND > 0) {
        dcols &= halt;
        halt &= ~dcols;
        if (dcols) {
          if (lane < 32u && ((dcols >> lane) & 1u)) {
            const uint32_t idx = n_def + (uint32_t)__builtin_popcount(dcols & ((1u << lane) - 1u));
            if (idx < p.defer_seg_cap) seg[idx] = toff;   // beyond: counted, flagged below
          }
          n_def += (uint32_t)__builtin_popcount(dcols);
        }
      }
      any1 &= halt;
      any0 &= halt;
      f_all += (uint32_t)__builtin_popcount(halt);
      f_1 += (uint32_t)__builtin_popcount(any1);
      f_2 += (uint32_t)__builtin_popcount(any1 & any0);
    }
    // No barrier here: the next group's /start writes only X (read before the
    // R-phase barrier), its R-phase writes PL after the barrier above (every
    // wave has finished this P-phase), and RED is rewritten only after the
    // next R-phase barrier, which wave 0 must reach.
  }
  if (wv == 0u) {
    if (KIND > 0 && n_def > p.defer_seg_cap) {   // segment overflow: extra trials dropped, launch flagged
      if (lane == 0) atomicOr(p.overflow, 1u);
      n_def = p.defer_seg_cap;
    }
    if (KIND > 0 && n_def) {                   // this workgroup's deferred trials -> the compact list
      __threadfence();
      uint32_t base = 0u;
      if (lane == 0) base = atomicAdd(p.defer_len, n_def);
      base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
      for (uint32_t i = lane; i < n_def; i += 64u) p.defer_list[base + i] = seg[i];
    }
    const uint32_t rb = 3u * (cont ? cont : 1u);   // bins 3R + v of the halting round R
    const uint32_t hc = lane == rb ? f_all - f_1 : (lane == rb + 1u ? f_1 - f_2 : (lane == rb + 2u ? f_2 : 0u));
    if (hc) atomicAdd(&lhist[lane], hc);
    if (lane == 0 && f_2) atomicAdd(&lhist[hist_len - 1u], f_2);
  }
  __syncthreads();
  flush_hist(lhist, p);
}

// Receiver tiles per block: big_nt(W).
static uint32_t coop_nt(const KParams &p) { return big_nt(p.W); }

static uint32_t coop_lds_bytes(const KParams &p, bool exp) {
  const uint32_t NT = coop_nt(p);
  return p.hist_bytes + (big_plane_words(p.W) + big_prop_words(p.W, NT)) * 64u * 4u * (exp ? 4u : 1u) + 16u * 4u * 4u;
}

// Expanded planes with four-tile blocks (W = 22..27), where one expansion
// serves only four products: x1.04 at N=1600 F=100, N=1700 F=300 and N=2048
// F=682; eight-tile blocks (W >= 28) measured within -2..+1 % either way, so
// they keep the packed words (profiles/r03-s3k_coop_exp_inproc.jsonl).
static bool coop_exp(const KParams &p) { return coop_lds_bytes(p, true) <= 160u * 1024u && coop_nt(p) == 4u; }

uint32_t mfma_coop_lds_bytes(const KParams &p) { return coop_lds_bytes(p, coop_exp(p)); }

// Waves per workgroup: 8 with eight-tile blocks (W >= 28: N=4096 F=1365 x1.04
// over 4 waves, F=0 equal), else 4 (W = 22..27: 8 waves x0.85-0.86, their
// four-tile blocks leave more registers and the CU takes more groups).
// BENOR_COOP_BW=4 / 8 forces one (validation knob: tests run both forms at
// every W, knob_value in benor_runtime.cpp).
uint32_t mfma_coop_block_waves(const KParams &p) {
  const uint32_t v = knob_u32("BENOR_COOP_BW", 0u);
  if (v == 4u || v == 8u) return v;
  return big_nt(p.W) == 8u ? 8u : 4u;
}

template <int KIND, int NT, int BW>
static int coop_occupancy(const KParams &p) {
  int n = 0;
  const void *fn = coop_exp(p) ? reinterpret_cast<const void *>(&benor_mfma_coop_kernel<KIND, NT, BW, true>)
                               : reinterpret_cast<const void *>(&benor_mfma_coop_kernel<KIND, NT, BW, false>);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 64 * BW, mfma_coop_lds_bytes(p)) != hipSuccess)
    n = 1;
  const int lds_fit = (int)lds_groups_per_cu(mfma_coop_lds_bytes(p));
  if (n > lds_fit) n = lds_fit;
  return n < 1 ? 1 : n;
}

int mfma_coop_blocks_per_cu(const KParams &p) {
  const bool nt8 = coop_nt(p) == 8u, bw8 = mfma_coop_block_waves(p) == 8u;
  const uint32_t k = p.G;
  if (nt8) {
    if (bw8) return k == 0 ? coop_occupancy<0, 8, 8>(p) : k == 1 ? coop_occupancy<1, 8, 8>(p) : coop_occupancy<2, 8, 8>(p);
    return k == 0 ? coop_occupancy<0, 8, 4>(p) : k == 1 ? coop_occupancy<1, 8, 4>(p) : coop_occupancy<2, 8, 4>(p);
  }
  if (bw8) return k == 0 ? coop_occupancy<0, 4, 8>(p) : k == 1 ? coop_occupancy<1, 4, 8>(p) : coop_occupancy<2, 4, 8>(p);
  return k == 0 ? coop_occupancy<0, 4, 4>(p) : k == 1 ? coop_occupancy<1, 4, 4>(p) : coop_occupancy<2, 4, 4>(p);
}

template <int KIND, int NT, int BW, bool EXP>
static hipError_t launch_coop_exp(const KParams &p, int grid, hipStream_t s) {
  const uint32_t lds = coop_lds_bytes(p, EXP);
  if (lds > 64u * 1024u) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&benor_mfma_coop_kernel<KIND, NT, BW, EXP>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((benor_mfma_coop_kernel<KIND, NT, BW, EXP>), dim3(grid), dim3(64 * BW), lds, s, p);
  return hipGetLastError();
}

template <int KIND, int NT, int BW>
static hipError_t launch_coop(const KParams &p, int grid, hipStream_t s) {
  return coop_exp(p) ? launch_coop_exp<KIND, NT, BW, true>(p, grid, s) : launch_coop_exp<KIND, NT, BW, false>(p, grid, s);
}

template <int KIND, int NT>
static hipError_t launch_coop_bw(const KParams &p, int grid, hipStream_t s) {
  return mfma_coop_block_waves(p) == 8u ? launch_coop<KIND, NT, 8>(p, grid, s) : launch_coop<KIND, NT, 4>(p, grid, s);
}

template <int KIND>
static hipError_t launch_coop_nt(const KParams &p, int grid, hipStream_t s) {
  return coop_nt(p) == 8u ? launch_coop_bw<KIND, 8>(p, grid, s) : launch_coop_bw<KIND, 4>(p, grid, s);
}

hipError_t launch_mfma_coop(const KParams &p, int grid, hipStream_t s) {
  if (p.W < 17u || p.W > kBigMaxW) return hipErrorInvalidValue;
  if (p.G == 0u) return launch_coop_nt<0>(p, grid, s);
  if (p.G == 1u) return launch_coop_nt<1>(p, grid, s);
  return launch_coop_nt<2>(p, grid, s);
}

}  // namespace benor
