// benor_lane_items.h -- lockstep kernel for short launches of small networks
// (2 <= m <= 24 live nodes, KIND 0: even m or ties possible; BASELINE
// configs[1] N=10, F=4 and the configs[0] shape N=5, F=1): every (trial,
// round) is one work item, and a wave runs 64 items at a time.
//
// Why items.  In lockstep every receiver of a trial hears the same inbox, so
// a round either halts the trial (no tie, m > F: every receiver decides the
// majority, node.ts:99-105) or leaves every receiver undecided -- after a
// tied R-phase (every proposal "?", node.ts:63-69) every receiver takes its
// coin (node.ts:110-111), so the next round's x plane is the round's coin
// word, a pure function of (seed, trial, round).  The rounds a trial will
// need are therefore known from its Philox words before any receiver counts,
// and the per-receiver work of each round can run anywhere.  A lane-per-trial
// kernel (benor_lane.h) keeps every lane on its own trial, so a wave runs as
// many rounds as its slowest trial; this kernel lays a trial's rounds out as
// items in a per-wave LDS ring and runs them 64 at a time on every lane:
//   * generator pass: each lane takes a fresh trial (or continues one that
//     has not halted after 4 rounds), draws its /start word and the coin
//     block of 4 rounds, and emits one item per round it needs, {x word |
//     round << 24, coin word} (rounds r0 .. r0+3, until the first round that
//     halts, or k_max);
//   * item passes: while 64 items are queued, each lane runs one item's round
//     -- every receiver's R-phase and P-phase tallies in its own opaque count
//     instruction (own_count / shift_in, exactly benor_lane.h's KIND 0 round
//     body) -- and the item that halts (every receiver decided) or reaches
//     k_max records the trial's outcome.
// The generator only decides how many items a trial gets; outcomes come from
// the items' own per-receiver tallies, so the histogram is the lane kernel's.
// Items carry no trial id: a round's result depends only on its x and coin
// words and r.  Outcome bins are counted per distinct bin of the batch with
// ballots (no contended LDS atomics).
#pragma once

#include "benor_lane.h"

namespace benor {

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <int MM>
__global__ void __launch_bounds__(256) benor_items_kernel(KParams p) {
  static_assert(MM >= 2 && MM <= (int)kItemsMaxM, "item word: x in 24 bits, round in 8");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = threadIdx.x >> 6;
  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint2 *Q = reinterpret_cast<uint2 *>(smem + p.hist_bytes) + (size_t)wv * kItemsRing;   // item ring
  for (uint32_t i = threadIdx.x; i < p.hist_len; i += blockDim.x) lhist[i] = 0u;
  __syncthreads();

  constexpr uint32_t live = (1u << MM) - 1u;
  constexpr uint32_t loT = (MM + 1) >> 1, hiT = MM >> 1;   // every vote binary: M = m (init_q = 0)
  const uint32_t F = p.F, k_max = p.k_max, hist_len = p.hist_len;
  const bool can_decide = (uint32_t)MM > F;
  const bool random_init = p.init_mode == BO_INIT_RANDOM;
  const uint32_t fixed1 = random_init ? 0u : (p.init_plane[0].z & live);
  const uint64_t gw = (uint64_t)blockIdx.x * kWavesPerBlock + wv;
  const uint64_t waves_total = (uint64_t)gridDim.x * kWavesPerBlock;
  const uint64_t trial_count = p.trial_count, trial_begin = p.trial_begin;

  // Outcome counters of the common bins 3r + v (r = 1..4, v = 0, 1), wave-
  // uniform: ballots and SALU popcounts per batch, no LDS traffic.
  uint32_t cnt[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};

  // One batch of n <= 64 queued items from `base`: lane l runs item base + l
  // (lanes >= n read a stale slot and record nothing).
  auto run_items = [&](uint32_t base, uint32_t n) {
    const bool v = lane < n;
    const uint2 it = Q[(base + lane) & (kItemsRing - 1u)];
    const uint32_t x1 = it.x & live, r = it.x >> 24, cwr = it.y;
    // R-phase (node.ts:46-82): c1 - loT (sign: p0), c1 - hiT - 1 (sign: not p1)
    uint32_t p0 = 0, np1 = 0;
#pragma unroll
    for (int c = MM - 1; c >= 0; --c) {
      const uint32_t s0 = own_count(x1, 0u - loT);
      shift_in(p0, s0);
      shift_in(np1, s0 + loT - hiT - 1u);
    }
    const uint32_t p1 = ~np1 & live;
    // P-phase (node.ts:83-113): a = c0 - F - 1 (not d0), b = c1 - F - 1 (not
    // d1), a - b (c1 > c0), b - a (c0 > c1)
    uint32_t nd0 = 0, nd1 = 0, gt1 = 0, gt0 = 0;
#pragma unroll
    for (int c = MM - 1; c >= 0; --c) {
      const uint32_t a = own_count(p0, 0u - (F + 1u)), b = own_count(p1, 0u - (F + 1u));
      shift_in(nd0, a);
      shift_in(nd1, b);
      shift_in(gt1, a - b);
      shift_in(gt0, b - a);
    }
    const uint32_t xn = nd0 & (~nd1 | gt1 | (~gt0 & cwr));
    const bool all_dec = (nd0 & nd1) == 0u;   // every live receiver decided (node.ts:99-105)
    // halt (auto-stop, node.ts:116-145) or k_max: the trial's outcome, bin
    // 3r + v (halted) or v (k_max), v = 1 / 0 / 2 (all x = 1 / all 0 / mixed)
    const bool rec = v && (all_dec || r >= k_max);
    const bool one = xn == live, zero = xn == 0u;
    const bool common = all_dec && r <= 4u && (one || zero);
    const uint64_t bc = ballot(rec && common), b1 = ballot(one);
#pragma unroll
    for (uint32_t rr = 1; rr <= 4u; ++rr) {
      const uint64_t br = ballot(r == rr) & bc;
      cnt[2u * rr - 2u] += (uint32_t)__builtin_popcountll(br & ~b1);
      cnt[2u * rr - 1u] += (uint32_t)__builtin_popcountll(br & b1);
    }
    if (rec && !common) {                     // rare: later rounds, k_max, split values
      const uint32_t val = one ? 1u : (zero ? 0u : 2u);
      atomicAdd(&lhist[all_dec ? 3u * r + val : val], 1u);
      if (all_dec && val == 2u) atomicAdd(&lhist[hist_len - 1u], 1u);
    }
  };

  bool cont = false;                          // this lane continues a trial from round r0
  uint32_t tlo = 0u, thi = 0u, xs = 0u, r0 = 1u;
  uint64_t next_j = 0;                        // the wave's next fresh trial: gw + next_j * waves_total
  uint32_t head = 0u, tail = 0u;              // ring positions (wave-uniform)
  for (;;) {
    // ---- generator pass (/start, node.ts:167-188, and the coins of node.ts:111)
    const uint64_t fm = ballot(!cont);
    bool act = cont;
    if (!cont) {
      const uint32_t rank = mbcnt64(fm);
      const uint64_t t = gw + (next_j + rank) * waves_total;
      if (t < trial_count) {
        const uint64_t tr = trial_begin + t;
        tlo = (uint32_t)tr;
        thi = (uint32_t)(tr >> 32);
        act = true;
        r0 = 1u;
        if (random_init) {
          uint32_t kk0 = (uint32_t)p.seed, kk1 = (uint32_t)(p.seed >> 32);
          asm volatile("" : "+s"(kk0), "+s"(kk1));
          xs = philox4x32_10(kk0, kk1, make_uint4(tlo, thi, 0u, kStreamInit << 24)).x & live;
        } else {
          xs = fixed1;
        }
      }
    }
    next_j += (uint64_t)__builtin_popcountll(fm);
    if (!__any(act)) break;
    uint4 cw = make_uint4(0u, 0u, 0u, 0u);
    if (act) {
      uint32_t kk0 = (uint32_t)p.seed, kk1 = (uint32_t)(p.seed >> 32);
      asm volatile("" : "+s"(kk0), "+s"(kk1));
      cw = coin_block(kk0, kk1, tlo, thi, 0u, r0);   // rounds r0 .. r0 + 3
    }
    // The rounds this trial runs in this pass (n = 0..4) and their x words,
    // as every receiver will find them: a tie sends every receiver to its
    // coin; otherwise every receiver proposed and voted the majority and
    // decides it (m > F: the trial halts) or adopts it (m <= F).
    const uint32_t cq[4] = {cw.x, cw.y, cw.z, cw.w};   // coin words of rounds r0 .. r0+3 (r0 = 1 mod 4)
    uint32_t xq[4], n = 0u;
    bool going = act;
    uint32_t x = xs;
#pragma unroll
    for (uint32_t q = 0; q < 4u; ++q) {
      xq[q] = x;
      const uint32_t r = r0 + q;
      if (going && r <= k_max) {
        n = q + 1u;
        const uint32_t c1 = (uint32_t)__builtin_popcount(x);
        const bool tie = 2u * c1 == (uint32_t)MM;
        if ((!tie && can_decide) || r >= k_max) going = false;
        else x = tie ? (cq[q] & live) : (2u * c1 > (uint32_t)MM ? live : 0u);
      } else {
        going = false;
      }
    }
    // ring positions: exclusive prefix of n over the lanes, bit by bit
    const uint64_t b0 = ballot(n & 1u), b1 = ballot(n & 2u), b2 = ballot(n & 4u);
    const uint32_t pos = mbcnt64(b0) + 2u * mbcnt64(b1) + 4u * mbcnt64(b2);
#pragma unroll
    for (uint32_t q = 0; q < 4u; ++q)
      if (q < n) Q[(tail + pos + q) & (kItemsRing - 1u)] = make_uint2(xq[q] | ((r0 + q) << 24), cq[q]);
    tail += (uint32_t)(__builtin_popcountll(b0) + 2 * __builtin_popcountll(b1) + 4 * __builtin_popcountll(b2));
    cont = going;                             // not halted after 4 rounds: continue next pass
    if (going) {
      xs = x;
      r0 += 4u;
    }
    // ---- item passes
    while (tail - head >= 64u) {
      run_items(head, 64u);
      head += 64u;
    }
  }
  if (tail != head) run_items(head, tail - head);
  if (lane == 0u) {
#pragma unroll
    for (uint32_t k = 0; k < 8u; ++k)
      if (cnt[k]) atomicAdd(&lhist[3u * (k / 2u + 1u) + (k & 1u)], cnt[k]);
  }

  __syncthreads();
  flush_hist(lhist, p);
}

template <int MM>
hipError_t launch_items_m(const KParams &p, int grid, hipStream_t s) {
  hipLaunchKernelGGL((benor_items_kernel<MM>), dim3(grid), dim3(64 * kWavesPerBlock), items_lds_bytes(p), s, p);
  return hipGetLastError();
}

}  // namespace benor
