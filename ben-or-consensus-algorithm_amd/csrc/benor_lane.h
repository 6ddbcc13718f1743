// benor_lane.h -- lockstep round loop for small networks (m <= 64 live nodes):
// one lane = one trial.  Instantiated by benor_lane_01_32.hip, benor_lane_33_48.hip
// and benor_lane_49_64.hip.
//
// Replaces the reference's POST /message handler (src/nodes/node.ts:43-163)
// for BASELINE configs C1 (N=5) and C2 (N=10, F=4 / F=5) and every other
// network of at most 32 live nodes.  A whole network fits one 32-bit word per
// bit plane, so each lane simulates one trial by itself:
//
//   * x1: bit c = live node c's x (compact order; a 32-bit word for m <= 32,
//     64-bit above); "?" only before round 1;
//   * R-phase (node.ts:46-82): every receiver c counts its own inbox, the m
//     live x messages -- c1 = popcount(x1) by that receiver's own opaque
//     v_bcnt_u32_b32 (asm volatile: the m identical lockstep counts of a trial
//     are never merged, SURVEY §7 "symmetry trap") -- and its proposal bit is
//     shifted into the proposal planes p1 / p0 by one compare and one add;
//   * P-phase (node.ts:83-158): every receiver counts p1 (and p0 unless every
//     vote is binary), decides / adopts / flips its coin, and its new x and
//     decided bits are shifted into the next planes;
//   * receivers are taken from c = m-1 down to 0, so after m shifts receiver c
//     sits at bit c again.
//
// Trials come from a per-wave queue exactly as in the packed design they
// replace: the wave's j-th trial is global trial gw + j * waves_total, so any
// launch split covers each trial id once.  The queue's Philox work -- the
// random initial values (one word of a block four trials share for m <= 32,
// two words of the trial's own block above) and, for m <= 32, the coin block of
// rounds 1-4 (benor_device.h coin_block) -- is drawn 64 trials per pass into
// an LDS ring; a lane that finishes its trial takes the next queue entry.
// Coins are needed only after a tied R-phase (all proposals "?", node.ts:63-69,
// 110-111); other coin blocks are drawn when a lane meets such a round.
// Outcomes go to the workgroup's LDS histogram, flushed once.
//
// KIND (fixed per plan): 2 = every vote count is odd and m > 2F, so every
// receiver decides in round 1 (x = majority); 1 = odd counts, m <= 2F (no tie
// can occur: no coin); 0 = general (even m, or "?" initial values).
#pragma once

#include <type_traits>

#include "benor_device.h"

namespace benor {

// One receiver's tally (node.ts:56-62, :92-98) over a 32- or 64-bit plane,
// offset by acc: popcount(plane) + acc (mod 2^32).  With acc = -T the sign bit
// of the result is (count < T), the receiver's comparison against a
// threshold in the same instruction.  asm volatile: the m identical lockstep
// counts of a trial are never merged (SURVEY §7 "symmetry trap").
__device__ __forceinline__ uint32_t own_count(uint32_t plane, uint32_t acc) {
  uint32_t r;
  asm volatile("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(plane), "v"(acc));
  return r;
}
__device__ __forceinline__ uint32_t own_count(uint64_t plane, uint32_t acc) {
  uint32_t r;
  asm volatile("v_bcnt_u32_b32 %0, %1, %2\n\tv_bcnt_u32_b32 %0, %3, %0" : "=&v"(r) : "v"((uint32_t)plane), "v"(acc),
               "v"((uint32_t)(plane >> 32)));
  return r;
}

// Receiver planes are built one receiver at a time, c = m-1 down to 0: the
// plane shifts left by one and takes the sign bit of the receiver's result
// (v_alignbit_b32: (plane << 1) | (r >> 31)), so after m receivers receiver c
// sits at bit c.
__device__ __forceinline__ void shift_in(uint32_t &plane, uint32_t r) { plane = __builtin_amdgcn_alignbit(plane, r, 31); }
__device__ __forceinline__ void shift_in(uint64_t &plane, uint32_t r) {
  const uint32_t lo = (uint32_t)plane, hi = (uint32_t)(plane >> 32);
  plane = ((uint64_t)__builtin_amdgcn_alignbit(hi, lo, 31) << 32) | __builtin_amdgcn_alignbit(lo, r, 31);
}

template <int MM, int KIND>
__global__ void __launch_bounds__(256) benor_lane_kernel(KParams p) {
  using Plane = std::conditional_t<(MM <= 32), uint32_t, uint64_t>;
  constexpr bool kWide = MM > 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = threadIdx.x >> 6;
  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint2 *iring = reinterpret_cast<uint2 *>(smem + p.hist_bytes + wv * p.wave_bytes);   // [128] init words
  uint4 *cring = reinterpret_cast<uint4 *>(iring + 128);                                // [128] coin blocks (m <= 32)
  for (uint32_t i = threadIdx.x; i < p.hist_len; i += blockDim.x) lhist[i] = 0u;
  __syncthreads();

  constexpr Plane live = MM == 8 * (int)sizeof(Plane) ? ~(Plane)0 : (((Plane)1 << MM) - 1);
  const uint32_t F = p.F, k_max = p.k_max, hist_len = p.hist_len;
  const bool random_init = p.init_mode == BO_INIT_RANDOM;
  const Plane fixed1 = random_init ? (Plane)0                                   // x1 words of a fixed init
                                   : (Plane)(p.init_plane[0].z | (kWide ? (uint64_t)p.init_plane[0].w << 32 : 0ull));
  const uint32_t M1 = MM - p.init_q;                               // binary votes in round 1
  const uint32_t mF = MM > F ? MM - F : 0u;
  const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
  const uint64_t gw = (uint64_t)blockIdx.x * kWavesPerBlock + wv;
  const uint64_t waves_total = (uint64_t)gridDim.x * kWavesPerBlock;

  uint64_t next_j = 0, filled = 0;
  bool need = true, act = false;
  Plane x1 = 0, dec = 0;
  uint32_t r = 0u, tlo = 0u, thi = 0u;
  uint4 cw = make_uint4(0u, 0u, 0u, 0u), cw1 = cw;                 // coin blocks (nodes 0-31, 32-63) of rounds
  uint32_t cg = 0u;                                                // 4(cg-1)+1 .. 4(cg-1)+4; cg = 0: none

  for (;;) {
    // ---- lanes whose trial ended take the next queue entries (/start, node.ts:167-188)
    const uint64_t needm = ballot(need);
    if (needm) {
      const uint32_t nn = (uint32_t)__builtin_popcountll(needm);
      if (next_j + nn > filled) {                                  // 64 queue entries per Philox pass
        const uint64_t j = filled + lane;
        const uint64_t t = gw + j * waves_total;
        if (t < p.trial_count) {
          const uint64_t tr = p.trial_begin + t;
          uint32_t kk0 = k0, kk1 = k1;
          asm volatile("" : "+s"(kk0), "+s"(kk1));
          if (random_init) {
            if constexpr (kWide) {
              const uint4 w = philox4x32_10(kk0, kk1, make_uint4((uint32_t)tr, (uint32_t)(tr >> 32), 0u, kStreamInit << 24));
              iring[j & 127u] = make_uint2(w.x, w.y);
            } else {                                               // m <= 32: the shared-block word
              iring[j & 127u] = make_uint2(init_word_small(kk0, kk1, tr), 0u);
            }
          }
          if (KIND == 0 && !kWide) cring[j & 127u] = coin_block(kk0, kk1, (uint32_t)tr, (uint32_t)(tr >> 32), 0u, 1u);
        }
        filled += 64u;
      }
      if (need) {
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(needm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)needm, 0u));
        const uint64_t j = next_j + below;
        const uint64_t t = gw + j * waves_total;
        act = t < p.trial_count;
        if (act) {
          const uint64_t tr = p.trial_begin + t;
          tlo = (uint32_t)tr;
          thi = (uint32_t)(tr >> 32);
          if (random_init) {
            const uint2 w = iring[j & 127u];
            x1 = (Plane)(w.x | (kWide ? (uint64_t)w.y << 32 : 0ull)) & live;
          } else {
            x1 = fixed1;
          }
          if (KIND == 0 && !kWide) cw = cring[j & 127u];
          cg = (KIND == 0 && !kWide) ? 1u : 0u;
          dec = 0;
          r = 0u;
        }
        need = false;
      }
      next_j += nn;
    }
    if (!__any(act)) break;
    if (!act) continue;

    ++r;
    // Every receiver c compares its own counts against the thresholds of
    // node.ts in the count instruction itself (own_count with acc = -T: sign
    // bit = count < T) and shifts the sign bits into receiver planes; the
    // decisions are then combined plane-wide, once per round.
    if (KIND == 2) {
      // M odd, m > 2F: proposal = majority, p0 = (c1 <= M/2) (node.ts:63-69);
      // every P-phase vote is binary and every receiver decides: x = 1 iff
      // c0 <= F, i.e. c1 >= m - F > F (node.ts:99-105)
      const uint32_t nT = 0u - (((r == 1u ? M1 : (uint32_t)MM) >> 1) + 1u);
      Plane p0 = 0;
#pragma unroll
      for (int c = MM - 1; c >= 0; --c) shift_in(p0, own_count(x1, nT));
      Plane nx = 0;
#pragma unroll
      for (int c = MM - 1; c >= 0; --c) shift_in(nx, own_count(p0, 0u - (F + 1u)));
      x1 = nx;
      dec = live;
    } else if (KIND == 1) {
      // M odd, m <= 2F: x = the vote majority (adopting it, node.ts:106-109, or
      // deciding it): c1 > m/2, i.e. c0 < (m+1)/2; decided iff c0 > F or
      // c1 > F, i.e. undecided iff m - F <= c0 <= F
      const uint32_t nT = 0u - (((r == 1u ? M1 : (uint32_t)MM) >> 1) + 1u);
      Plane p0 = 0;
#pragma unroll
      for (int c = MM - 1; c >= 0; --c) shift_in(p0, own_count(x1, nT));
      Plane nx = 0, lo = 0, hi = 0;                                  // lo: c0 < m - F; hi: c0 > F
#pragma unroll
      for (int c = MM - 1; c >= 0; --c) {
        const uint32_t s = own_count(p0, 0u - (uint32_t)((MM + 1) / 2));   // c0 - (m+1)/2
        shift_in(nx, s);
        shift_in(lo, s + (uint32_t)((MM + 1) / 2) - mF);             // c0 - (m - F)
        shift_in(hi, F - (s + (uint32_t)((MM + 1) / 2)));            // F - c0
      }
      x1 = nx;
      dec |= (lo | hi) & live;
    } else {
      // General: c0 = M - c1 (M binary votes); p1 = c1 > c0, p0 = c0 > c1,
      // else "?" (node.ts:63-69)
      const uint32_t M = r == 1u ? M1 : (uint32_t)MM;
      const uint32_t hiT = M >> 1, loT = (M + 1u) >> 1;
      Plane p0 = 0, np1 = 0;
#pragma unroll
      for (int c = MM - 1; c >= 0; --c) {
        const uint32_t s0 = own_count(x1, 0u - loT);                // c1 - loT: sign = p0
        shift_in(p0, s0);
        shift_in(np1, s0 + loT - hiT - 1u);                           // c1 - hiT - 1: sign = not p1
      }
      const Plane p1 = ~np1 & live;
      // Coins (node.ts:111) are flipped only after a tied R-phase (every
      // proposal "?"): this lane's coin block for round r is drawn then, unless
      // it holds it already (rounds 1-4 of m <= 32 come from the ring).
      const uint32_t g1 = ((r - 1u) >> 2) + 1u;
      if (2u * (uint32_t)__builtin_popcountll((uint64_t)x1) == M && cg != g1) {
        uint32_t kk0 = k0, kk1 = k1;
        asm volatile("" : "+s"(kk0), "+s"(kk1));
        cw = coin_block(kk0, kk1, tlo, thi, 0u, r);
        if (kWide) cw1 = coin_block(kk0, kk1, tlo, thi, 32u, r);
        cg = g1;
      }
      const Plane cwr = (Plane)(coin_word_v(cw, r) | (kWide ? (uint64_t)coin_word_v(cw1, r) << 32 : 0ull));
      // P-phase (node.ts:88-113), per receiver: a = c0 - F - 1 (sign: not d0),
      // b = c1 - F - 1 (sign: not d1), a - b = c0 - c1 (sign: c1 > c0),
      // b - a (sign: c0 > c1)
      Plane nd0 = 0, nd1 = 0, gt1 = 0, gt0 = 0;
#pragma unroll
      for (int c = MM - 1; c >= 0; --c) {
        const uint32_t a = own_count(p0, 0u - (F + 1u)), b = own_count(p1, 0u - (F + 1u));
        shift_in(nd0, a);
        shift_in(nd1, b);
        shift_in(gt1, a - b);
        shift_in(gt0, b - a);
      }
      // x = 0 if d0, else 1 if d1, else the majority (node.ts:106-109), else
      // the coin (node.ts:111); decided = d0 or d1 (node.ts:99-105)
      x1 = nd0 & (~nd1 | gt1 | (~gt0 & cwr));
      dec |= ~(nd0 & nd1) & live;
    }

    // ---- halt: every live node decided (auto-stop, node.ts:116-145) or k_max
    const bool all_dec = dec == live;
    if (all_dec || r >= k_max) {
      const uint32_t v = x1 == live ? 1u : (x1 == 0 ? 0u : 2u);
      atomicAdd(&lhist[all_dec ? r * 3u + v : v], 1u);
      if (all_dec && v == 2u) atomicAdd(&lhist[hist_len - 1u], 1u);
      if (p.rounds_out) *p.rounds_out = all_dec ? r : 0u;
      if (p.node_out) {                                            // GET /getState (node.ts:197-199)
        for (uint32_t c = 0; c < (uint32_t)MM; ++c) {
          bo_node_state ns;
          ns.killed = 0;
          ns.x = (int8_t)((x1 >> c) & 1u);
          ns.decided = (int8_t)((dec >> c) & 1u);
          ns.pad = 0;
          ns.k = (int32_t)r + 1;                                   // node.ts:147
          p.node_out[p.live_ids[c]] = ns;
        }
      }
      act = false;
      need = true;
    }
  }

  __syncthreads();
  flush_hist(lhist, p);
}

template <int MM, int KIND>
static hipError_t launch_lane_k(const KParams &p, int grid, hipStream_t s) {
  hipLaunchKernelGGL((benor_lane_kernel<MM, KIND>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  return hipGetLastError();
}

template <int MM>
hipError_t launch_lane_m(const KParams &p, int grid, hipStream_t s) {
  if constexpr ((MM & 1) != 0) {
    if (p.G == 2u) return launch_lane_k<MM, 2>(p, grid, s);
    if (p.G == 1u) return launch_lane_k<MM, 1>(p, grid, s);
  }
  return launch_lane_k<MM, 0>(p, grid, s);
}

}  // namespace benor
