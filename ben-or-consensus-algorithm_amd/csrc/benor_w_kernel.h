// benor_w_kernel.h -- the W-specialised lockstep kernel (W = ceil(m/64) <= 32
// receiver groups, fully unrolled) and its launcher.  Instantiated for W ranges
// in benor_w_*.hip so the unrolled instantiations compile in parallel.
#pragma once

#include "benor_device.h"

namespace benor {

// STATE: the network API's single-trial launch that also reports per-node
// state and the halting round (GET /getState); the batch path is compiled
// without that code, which keeps its register allocation free of it.
constexpr int kPairMaxW = 8;               // W kernel: pair trials' round 1 up to this W

// Trials whose round 1 runs interleaved (K).  A small-W round is a handful of
// words, so more independent trials hide the ballot -> s_nop -> v_bcnt and LDS
// latencies.  Odd-only kernels carry no even-M code and take the larger K.
// K divides the init batch TB = 64 / ceil(W/2) where it can.  v19 A/B
// (profiles/r01-v19_ab_interleave_k.jsonl): odd W=1 +27 %, W=2 +10 %, W=3 +7 %,
// W=4 +2 %; even W=1 +8 %, W=2 +4 %, W=3 +2 %, W=4 +1.5 %; larger K spills.
constexpr int interleave_k(int W, bool odd_only) {
  if (odd_only) return W <= 4 ? 8 : (W <= 6 ? 3 : (W <= 16 ? 2 : 1));   // W >= 2 (m > 64)
  return W <= 2 ? 8 : (W <= 4 ? 4 : (W <= 6 ? 3 : (W <= kPairMaxW ? 2 : 1)));
}

// ODD_ONLY: every round's binary vote count is odd (m odd, and an even number
// of "?" initial values) -- the even-M code is not compiled, which frees the
// registers it would hold (batch path only).
// One interleaved trial's round-1 outcome in SALU only (the compiler turns
// the equivalent selects into VALU lane masks): a trial with some undecided
// receiver (rest != 0) is flagged in `slow` for a re-run; otherwise it counts
// in f1 if some x = 1 and in f2 if both values occur.
__device__ __forceinline__ void count_halt(uint64_t rest, uint64_t any0, uint64_t any1, uint32_t bit,
                                           uint32_t &f1, uint32_t &f2, uint32_t &slow) {
  uint64_t t;
  uint32_t b;
  asm volatile(
      "s_cmp_eq_u64 %[rest], 0\n\t"
      "s_cselect_b64 %[t], %[a1], 0\n\t"      // t = halted ? any1 : 0
      "s_cselect_b32 %[b], 0, %[bit]\n\t"     // b = halted ? 0 : bit
      "s_or_b32 %[slow], %[slow], %[b]\n\t"
      "s_cmp_lg_u64 %[t], 0\n\t"
      "s_addc_u32 %[f1], %[f1], 0\n\t"
      "s_cmp_lg_u64 %[a0], 0\n\t"
      "s_cselect_b64 %[t], %[t], 0\n\t"
      "s_cmp_lg_u64 %[t], 0\n\t"
      "s_addc_u32 %[f2], %[f2], 0"
      : [f1] "+s"(f1), [f2] "+s"(f2), [slow] "+s"(slow), [t] "=&s"(t), [b] "=&s"(b)
      : [rest] "s"(rest), [a0] "s"(any0), [a1] "s"(any1), [bit] "s"(bit)
      : "scc");
}

// The same for a trial where every receiver decided (odd vote count and
// m > 2F, decide_k's SURE case): it halts, and every live node holds a value,
// so some x = 0 or some x = 1.  f1 += [some 1]; f2 += [some 0] + [some 1],
// and the caller takes 1 off f2 per trial: [both] = [some 0] + [some 1] - 1.
__device__ __forceinline__ void count_sure(uint64_t any0, uint64_t any1, uint32_t &f1, uint32_t &f2) {
  asm volatile(
      "s_cmp_lg_u64 %[a1], 0\n\t"
      "s_addc_u32 %[f1], %[f1], 0\n\t"
      "s_cmp_lg_u64 %[a1], 0\n\t"
      "s_addc_u32 %[f2], %[f2], 0\n\t"
      "s_cmp_lg_u64 %[a0], 0\n\t"
      "s_addc_u32 %[f2], %[f2], 0"
      : [f1] "+s"(f1), [f2] "+s"(f2)
      : [a0] "s"(any0), [a1] "s"(any1)
      : "scc");
}

template <int W, bool STATE, bool ODD_ONLY = false>
__global__ void __launch_bounds__(256) benor_lockstep_w_kernel(KParams p) {
  constexpr int NPH = (W + 1) / 2;          // Philox blocks per trial (2 plane words each)
  constexpr int TB = 64 / NPH;              // trials per init batch
  constexpr int WP = 2 * NPH;               // x1 words per plane row, padded to 16 bytes
  constexpr int K = interleave_k(W, ODD_ONLY);   // trials whose round 1 runs interleaved
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // uniform: scalar trial loop
  // Only the round loop's own scalars are kept in registers.  What a rare
  // path needs (Philox key, trial id base) sits in a small LDS
  // parameter block and is re-read where it is used, so the register
  // allocator never holds -- and spills -- a kernarg tuple across the
  // trial loop.
  uint32_t m = p.m, F = p.F, k_max = p.k_max, hist_len = p.hist_len;
  // trial offsets within the launch are 32-bit (the host splits launches at 2^31)
  uint32_t trial_count = (uint32_t)p.trial_count;
  const bool listed = p.trial_list_len != nullptr;
  if (listed) {                    // trial-list mode: the list's length, set on the device
    const uint32_t n = *p.trial_list_len;
    trial_count = n < trial_count ? n : trial_count;
  }
  asm volatile("" : "+s"(m), "+s"(F), "+s"(k_max), "+s"(hist_len), "+s"(trial_count));

  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint2 *ring = reinterpret_cast<uint2 *>(smem + p.hist_bytes + wv * p.wave_bytes);   // [TB][WP] x1 words
  uint2 *X = ring + TB * WP;       // [WP] final x1 plane (GET /getState only)
  uint2 *D = X + WP;               // [WP] sticky decided bits, kept only while some receiver is undecided
  // parameter block: [0,1] Philox key (seed), [2,3] trial_begin, [4,5] trial list (or 0)
  uint32_t *keys = reinterpret_cast<uint32_t *>(smem + p.hist_bytes - kParamBytes);

  for (uint32_t i = threadIdx.x; i < hist_len; i += blockDim.x) lhist[i] = 0u;
  if (threadIdx.x == 0) {
    keys[0] = (uint32_t)p.seed;
    keys[1] = (uint32_t)(p.seed >> 32);
    keys[2] = (uint32_t)p.trial_begin;
    keys[3] = (uint32_t)(p.trial_begin >> 32);
    keys[4] = (uint32_t)(uintptr_t)p.trial_list;
    keys[5] = (uint32_t)((uintptr_t)p.trial_list >> 32);
  }
  if (p.init_mode != BO_INIT_RANDOM && lane < (uint32_t)W) {
    const uint4 q = p.init_plane[lane];
    ring[lane] = make_uint2(q.z, q.w);
  }
  __syncthreads();

  const uint32_t waves_total = gridDim.x * kWavesPerBlock;
  const uint64_t tailm = group_mask(W - 1, m);
  const bool random_init = p.init_mode == BO_INIT_RANDOM;
  const uint32_t m_first = m - p.init_q;      // binary-valued senders in round 1 ("?" excluded)

  uint32_t hc = 0;                            // this wave's outcome counts of bins 0..63, lane = bin
  // Interleaved round-1 halts (R = 1, every receiver decided; bins 3 + v) are
  // counted in three scalars -- halts, halts with some x = 1, halts with both
  // values -- and folded into `hc` once at the end: no per-trial VALU, no branch.
  uint32_t f_all = 0, f_1 = 0, f_2 = 0;
  for (uint32_t base = blockIdx.x * kWavesPerBlock + wv; base < trial_count; base += waves_total * TB) {
    // ---- /start (node.ts:167-188): round-1 x planes of TB trials at once.
    if (random_init) {
      const uint32_t s = lane / NPH, b = lane - s * NPH;
      const uint32_t t = base + s * waves_total;
      if (s < (uint32_t)TB && t < trial_count) {
        const uint64_t trial = trial_id(keys, t);
        const uint2 kk = lds_keys(keys);           // keep the round keys out of long-lived SGPRs
        const uint4 r = philox4x32_10(kk.x, kk.y, make_uint4((uint32_t)trial, (uint32_t)(trial >> 32), b, kStreamInit << 24));
        const uint64_t v0 = group_mask(2u * b, m), v1 = group_mask(2u * b + 1u, m);
        const uint64_t x1a = ((uint64_t)r.y << 32 | r.x) & v0, x1b = ((uint64_t)r.w << 32 | r.z) & v1;
        reinterpret_cast<uint4 *>(ring + s * WP)[b] =
            make_uint4((uint32_t)x1a, (uint32_t)(x1a >> 32), (uint32_t)x1b, (uint32_t)(x1b >> 32));
      }
    }
    // One trial's outcome: bins 0..63 (undecided, and halting rounds <= 20) in
    // lane `bin` of the wave's counter (one VALU op), the rest as LDS atomics.
    auto record = [&](uint64_t any0, uint64_t any1, uint32_t R, bool all_dec) {
      const uint32_t v = (any0 && any1) ? 2u : (any1 ? 1u : 0u);
      const uint32_t bin = all_dec ? (R * 3u + v) : v;
      if (bin < 64u) hc += (lane == bin) ? 1u : 0u;
      else if (lane == 0) atomicAdd(&lhist[bin], 1u);
      if (all_dec && v == 2u && lane == 0) atomicAdd(&lhist[hist_len - 1u], 1u);
    };
    // One whole trial, round after round.
    auto single = [&](int s, uint32_t t) {
      // ---- round-1 R-phase tallies over the /start broadcast (node.ts:167-188)
      uint32_t c1r[W];
      tally_x1<W>(random_init ? ring + s * WP : ring, c1r);
      uint64_t any0 = 0, any1 = 0;            // final round's x: some live node 0 / some 1
      uint32_t R = 0, M = m_first;
      bool all_dec = false, have_hist = false;
      for (uint32_t r = 1;; ++r) {
        // ---- R-phase ("proposal phase", node.ts:46-82) proposals from c1 (c0 = M - c1)
        // fused with the P-phase ("voting phase", node.ts:83-158) tallies.  With an
        // odd number M of binary votes c0 == c1 is impossible, so "c0 > c1" is the
        // complement of "c1 > c0" and costs no second compare (ODD: one copy of the
        // phase per parity, no branch inside it).
        uint32_t a0[1][W], a1[1][W];
        uint64_t rest_any[1], any0_[1], any1_[1];
        auto& c1v = reinterpret_cast<uint32_t(&)[1][W]>(c1r);
        const bool odd = ODD_ONLY || (M & 1u);
        if (odd) {
          p_phase_k<true, W, 1>(c1v, M, tailm, a0, a1);
          if (m > 2u * F) decide_k<true, true, W, 1>(a0, a1, m, F, tailm, rest_any, any0_, any1_);
          else decide_k<true, false, W, 1>(a0, a1, m, F, tailm, rest_any, any0_, any1_);
        } else if constexpr (!ODD_ONLY) {
          p_phase_k<false, W, 1>(c1v, M, tailm, a0, a1);
          decide_k<false, false, W, 1>(a0, a1, m, F, tailm, rest_any, any0_, any1_);
        }
        R = r;                                                        // node.ts:147  k = r + 1
        any0 = any0_[0];
        any1 = any1_[0];
        // ---- when every live receiver decides in this round the trial halts
        // (decided is sticky) and x = the decided value, so neither the
        // adopt/coin branch nor the next round's planes are needed.
        if (!rest_any[0] && !STATE) {
          all_dec = true;                                             // all-decided auto-stop
          break;
        }
        // ---- some receiver did not decide: adopt / coin (node.ts:106-113), the
        // sticky decided history (LDS, only on this path), and the next round's
        // R-phase tallies fused with the new x ballots (no staged plane).
        const bool more = r < k_max;
        uint64_t undone = 0;
        uint32_t sx = 0, sd = 0;
        any0 = 0;
        any1 = 0;
        Unroll<W>::run([&](auto gi) {
          constexpr int g = decltype(gi)::value;
          const uint64_t vm = (g == W - 1) ? tailm : ~0ull;
          const uint32_t Fg = F + (uint32_t)g;
          // ODD round: no c0 tally was made; c0 = m - c1 (all votes binary), bias g
          uint32_t a0g = (m + 2u * (uint32_t)g) - a1[0][g];
          if constexpr (!ODD_ONLY) a0g = odd ? a0g : a0[0][g];
          const uint32_t a1g = a1[0][g];
          const uint64_t d0 = vcmp_gt(a0g, Fg) & vm;
          const uint64_t d1 = vcmp_gt(a1g, Fg) & vm & ~d0;
          const uint64_t rest = vm & ~(d0 | d1);
          uint64_t x1 = d1;
          if (rest) {
            const uint64_t ad1 = ballot_s(a1g > a0g) & rest;             // node.ts:108-109
            const uint64_t tie = ballot_s(a1g == a0g) & rest;            // node.ts:110-111
            x1 |= ad1;
            if (tie) {                                                  // node.ts:111
              const uint64_t trial = trial_id(keys, t);
              x1 |= coin_ballot(keys, (uint32_t)trial, (uint32_t)(trial >> 32), g, r, tie);
            }
          }
          uint64_t dg = d0 | d1;
          if (have_hist) {
            const uint2 h = D[g];
            dg |= (uint64_t)sgpr32(h.y) << 32 | sgpr32(h.x);
          }
          sd = writelane<2 * g>(sd, (uint32_t)dg);
          sd = writelane<2 * g + 1>(sd, (uint32_t)(dg >> 32));
          undone |= vm & ~dg;
          any1 |= x1;
          any0 |= vm & ~x1;
          asm volatile("" : "+s"(undone), "+s"(any0), "+s"(any1));   // fold per group (as in the decisions)
          const uint32_t xl = sgpr32((uint32_t)x1), xh = sgpr32((uint32_t)(x1 >> 32));
          if (more) {                                                 // round r+1 R-phase (node.ts:149-157)
            if constexpr (g == 0) {
              Unroll<W>::run([&](auto hi) {
                constexpr int h = decltype(hi)::value;
                c1r[h] = tally_first_s<h>(xl);
              });
            } else {
#pragma unroll
              for (int h = 0; h < W; ++h) c1r[h] = tally_s(xl, c1r[h]);
            }
#pragma unroll
            for (int h = 0; h < W; ++h) c1r[h] = tally_s(xh, c1r[h]);
          }
          if constexpr (STATE) {
            sx = writelane<2 * g>(sx, xl);
            sx = writelane<2 * g + 1>(sx, xh);
          }
        });
        if (lane < 2u * W) {
          reinterpret_cast<uint32_t *>(D)[lane] = sd;
          if (STATE) reinterpret_cast<uint32_t *>(X)[lane] = sx;
        }
        have_hist = true;
        M = m;
        all_dec = undone == 0;
        if (all_dec || !more) break;
      }
      // ---- outcome
      record(any0, any1, R, all_dec);
      if constexpr (STATE) {
        uint32_t *rounds_out = p.rounds_out;
        if (lane == 0 && rounds_out) *rounds_out = all_dec ? R : 0u;
      }
      bo_node_state *node_out = STATE ? p.node_out : nullptr;
      if (STATE && node_out) {                                               // GET /getState (node.ts:197-199)
        Unroll<W>::run([&](auto gi) {
          constexpr int g = decltype(gi)::value;
          const uint32_t c = g * 64u + lane;
          if (c < m) {
            const uint2 q = X[g], d = D[g];
            bo_node_state ns;
            ns.killed = 0;
            ns.x = (int8_t)(((lane < 32u ? q.x : q.y) >> (lane & 31u)) & 1u);
            ns.decided = (int8_t)(((lane < 32u ? d.x : d.y) >> (lane & 31u)) & 1u);
            ns.pad = 0;
            ns.k = (int32_t)R + 1;
            node_out[p.live_ids[c]] = ns;
          }
        });
      }
    };
    for (int s = 0; s < TB;) {
      const uint32_t t = base + (uint32_t)s * waves_total;
      if (t >= trial_count) break;
      uint32_t slow = 1u, nk = 1u;              // trials (bit k: s + k) to run alone; trials consumed
      if constexpr (K > 1 && !STATE) {
        // (not in trial-list mode: the matrix-core kernel's deferred trials
        // never halt in round 1, so the interleaved pass would only be redone)
        if (!listed && s + K - 1 < TB && t + (uint32_t)(K - 1) * waves_total < trial_count) {
          // ---- round 1 of K trials interleaved; a trial that does not halt in
          // round 1 (some receiver undecided) is re-run alone from round 1.
          uint32_t c1[K][W], a0[K][W], a1[K][W];
          Unroll<K>::run([&](auto ki) {
            constexpr int k = decltype(ki)::value;
            tally_x1<W>(random_init ? ring + (s + k) * WP : ring, c1[k]);
          });
          uint64_t rest_any[K], any0[K], any1[K];
          slow = 0u;
          nk = K;
          auto count_all = [&]() {
            f_all += K;                         // minus the re-run trials, below
            Unroll<K>::run([&](auto ki) {
              constexpr int k = decltype(ki)::value;
              count_halt(rest_any[k], any0[k], any1[k], 1u << k, f_1, f_2, slow);
            });
            f_all -= (uint32_t)__builtin_popcount(slow);
          };
          if (ODD_ONLY || (m_first & 1u)) {
            p_phase_k<true, W, K>(c1, m_first, tailm, a0, a1);
            if (m > 2u * F) {                   // every receiver decides: all K trials halt
              decide_k<true, true, W, K>(a0, a1, m, F, tailm, rest_any, any0, any1);
              f_all += K;
              f_2 -= K;
              Unroll<K>::run([&](auto ki) {
                constexpr int k = decltype(ki)::value;
                count_sure(any0[k], any1[k], f_1, f_2);
              });
            } else {
              decide_k<true, false, W, K>(a0, a1, m, F, tailm, rest_any, any0, any1);
              count_all();
            }
          } else if constexpr (!ODD_ONLY) {
            p_phase_k<false, W, K>(c1, m_first, tailm, a0, a1);
            decide_k<false, false, W, K>(a0, a1, m, F, tailm, rest_any, any0, any1);
            count_all();
          }
        }
      }
      for (; slow; slow &= slow - 1u) {         // one call site: the whole-trial loop is inlined once
        const uint32_t k = (uint32_t)__builtin_ctz(slow);
        single(s + (int)k, t + k * waves_total);
      }
      s += (int)nk;
    }
  }

  hc += lane == 3u ? f_all - f_1 : (lane == 4u ? f_1 - f_2 : (lane == 5u ? f_2 : 0u));   // R = 1: v = 0, 1, 2
  if (hc) atomicAdd(&lhist[lane], hc);
  if (lane == 0 && f_2) atomicAdd(&lhist[hist_len - 1u], f_2);                     // disagreement counter
  __syncthreads();
  flush_hist(lhist, p);
}

// The runtime's grid asks for 8 workgroups per CU whatever the occupancy;
// workgroups that do not fit queue behind the resident ones.  Capping the grid
// at the resident count was measured slower (-0.5..-4 %).
template <int W>
hipError_t launch_w(const KParams &p, int grid, hipStream_t s) {
  const bool state = p.node_out || p.rounds_out;
  const bool odd_only = (p.m & 1u) && !(p.init_q & 1u);   // M = m - init_q in round 1, m after
  if (state)
    hipLaunchKernelGGL((benor_lockstep_w_kernel<W, true>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  else if (odd_only)
    hipLaunchKernelGGL((benor_lockstep_w_kernel<W, false, true>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  else
    hipLaunchKernelGGL((benor_lockstep_w_kernel<W, false>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  return hipGetLastError();
}

}  // namespace benor
