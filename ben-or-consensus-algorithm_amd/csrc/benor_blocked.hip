// benor_blocked.hip -- the blocked lockstep kernel (32 < W <= 64 receiver
// groups, processed in NB runtime blocks of G = ceil(W/NB) in 11..22 groups,
// NB chosen by plan_geometry for the fewest padded groups) and its launcher.
#include "benor_device.h"

namespace benor {

// --------------------------------------------- blocked kernel (1024 < m <= 4096)
// Receiver groups are processed in NB blocks of G (see plan_geometry); the
// record loop over the W plane words is a runtime loop.  Per-lane `decided`
// bits live in the wave's LDS slice (one word per block).  Otherwise as the
// W-specialised kernel.
// Word-major tallies: each plane word is applied to all G receiver groups
// before the next word, so consecutive v_bcnt are independent (tally_ordered
// keeps that order; see benor_device.h).
template <int G>
__device__ __forceinline__ void add_word(uint32_t word, uint32_t (&a)[G]) {
#pragma unroll
  for (int g = 0; g < G; ++g) a[g] = tally_ordered(word, a[g]);
}

// P-phase tally over W {p0.lo, p0.hi, p1.lo, p1.hi} records (runtime W).
template <int G>
__device__ __forceinline__ void tally_groups(const uint4 *__restrict__ plane, uint32_t W, uint32_t (&a0)[G],
                                             uint32_t (&a1)[G]) {
  const uint4 q = plane[0];
  Unroll<G>::run([&](auto gi) {
    constexpr int g = decltype(gi)::value;
    a0[g] = tally_first<g>(q.x);
  });
  Unroll<G>::run([&](auto gi) {
    constexpr int g = decltype(gi)::value;
    a1[g] = tally_first<g>(q.z);
  });
  add_word<G>(q.y, a0);
  add_word<G>(q.w, a1);
  for (uint32_t w = 1; w < W; ++w) {
    const uint4 u = plane[w];
    add_word<G>(u.x, a0);
    add_word<G>(u.z, a1);
    add_word<G>(u.y, a0);
    add_word<G>(u.w, a1);
  }
}

// c1-only tally over the W words of an x1-style plane (runtime W, pairs of
// groups per 16-byte read; WP = W rounded up to even, padding words zero).
template <int G>
__device__ __forceinline__ void tally_groups_x1(const uint2 *__restrict__ plane, uint32_t W, uint32_t (&a1)[G]) {
  const uint4 *q4 = reinterpret_cast<const uint4 *>(plane);
  const uint4 q = q4[0];
  Unroll<G>::run([&](auto gi) {
    constexpr int g = decltype(gi)::value;
    a1[g] = tally_first<g>(q.x);
  });
  add_word<G>(q.y, a1);
  add_word<G>(q.z, a1);
  add_word<G>(q.w, a1);
  const uint32_t np = (W + 1u) >> 1;
  for (uint32_t w = 1; w < np; ++w) {
    const uint4 u = q4[w];
    add_word<G>(u.x, a1);
    add_word<G>(u.y, a1);
    add_word<G>(u.z, a1);
    add_word<G>(u.w, a1);
  }
}

// One block's R-phase proposals (node.ts:63-69) from the receivers' c1
// counts, staged as {p0.lo, p0.hi, p1.lo, p1.hi} records for the P-phase
// tallies of every block.  ODD: an odd number of binary votes cannot tie,
// so p0 is the complement of p1 (one compare per group).
template <bool ODD, int G>
__device__ __forceinline__ uint2 stage_proposals(const uint32_t (&a1)[G], uint32_t b, uint32_t m, uint32_t M) {
  const uint32_t hi_t = M >> 1, lo_t = (M + 1u) >> 1;
  uint32_t st = 0, st2 = 0;                     // records of groups 0..15 and 16..G-1 (4 lanes each)
  Unroll<G>::run([&](auto gi) {
    constexpr int g = decltype(gi)::value;
    const uint64_t vm = group_mask(b * G + g, m);
    const uint64_t p1 = vcmp_gt(a1[g], hi_t + (uint32_t)g) & vm;          // c1 > c0  (node.ts:65-66)
    const uint64_t p0 = ODD ? (vm & ~p1)                                   // c0 > c1  (node.ts:63-64)
                            : (vcmp_lt(a1[g], lo_t + (uint32_t)g) & vm);   // else "?"
    if constexpr (g < 16) st = stage4<g>(st, p0, p1);
    else st2 = stage4<g - 16>(st2, p0, p1);
  });
  return make_uint2(st, st2);
}

template <int G, bool STATE>
__global__ void __launch_bounds__(256) benor_lockstep_blocked_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // scalar trial loop
  // Round-loop scalars in registers; the rest re-read where used (as the W kernel).
  uint32_t m = p.m, F = p.F, W = p.W, NB = p.nblocks, k_max = p.k_max, hist_len = p.hist_len;
  uint32_t trial_count = (uint32_t)p.trial_count;     // launches are split at 2^31 trials
  if (p.trial_list_len) {                    // trial-list mode (as the W kernel): the list's length
    const uint32_t n = *p.trial_list_len;
    trial_count = n < trial_count ? n : trial_count;
  }
  asm volatile("" : "+s"(m), "+s"(F), "+s"(W), "+s"(NB));
  asm volatile("" : "+s"(k_max), "+s"(hist_len), "+s"(trial_count));
  const uint32_t nph = (W + 1u) >> 1, tb = 64u / nph, WP = 2u * nph;
  const uint32_t XW = ((NB * G > WP ? NB * G : WP) + 1u) & ~1u;   // x1 words of the staged plane (even, padding zero)
  const uint32_t tail_n = m - (W - 1u) * 64u;          // live receivers in the last group

  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint32_t *keys = reinterpret_cast<uint32_t *>(smem + p.hist_bytes - kParamBytes);   // see the W kernel
  uint2 *ring = reinterpret_cast<uint2 *>(smem + p.hist_bytes + wv * p.wave_bytes);   // [tb][WP] x1 words
  uint2 *X = ring + tb * WP;                                                            // [XW]
  uint4 *P = reinterpret_cast<uint4 *>(X + XW);                                        // [NB*G]
  uint32_t *D = reinterpret_cast<uint32_t *>(P + NB * G);                               // [NB][64] decided bits

  for (uint32_t i = threadIdx.x; i < hist_len; i += blockDim.x) lhist[i] = 0u;
  if (threadIdx.x == 0) {
    keys[0] = (uint32_t)p.seed;
    keys[1] = (uint32_t)(p.seed >> 32);
    keys[2] = (uint32_t)p.trial_begin;
    keys[3] = (uint32_t)(p.trial_begin >> 32);
    keys[4] = (uint32_t)(uintptr_t)p.trial_list;
    keys[5] = (uint32_t)((uintptr_t)p.trial_list >> 32);
  }
  if (p.init_mode != BO_INIT_RANDOM)
    for (uint32_t w = lane; w < WP; w += 64u) {
      const uint4 q = w < W ? p.init_plane[w] : make_uint4(0, 0, 0, 0);
      ring[w] = make_uint2(q.z, q.w);
    }
  for (uint32_t w = lane; w < XW; w += 64u) X[w] = make_uint2(0u, 0u);
  __syncthreads();

  const uint32_t waves_total = gridDim.x * kWavesPerBlock;
  const bool random_init = p.init_mode == BO_INIT_RANDOM;
  const uint32_t m_first = m - p.init_q;

  uint32_t hc = 0;                            // this wave's outcome counts of bins 0..63, lane = bin
  for (uint32_t base = blockIdx.x * kWavesPerBlock + wv; base < trial_count; base += waves_total * tb) {
    if (random_init) {                       // /start (node.ts:167-188), tb trials per Philox pass
      const uint32_t s = lane / nph, bk = lane - s * nph;
      const uint32_t t = base + s * waves_total;
      if (s < tb && t < trial_count) {
        const uint64_t trial = trial_id(keys, t);
        const uint2 kk = lds_keys(keys);
        const uint4 r = philox4x32_10(kk.x, kk.y, make_uint4((uint32_t)trial, (uint32_t)(trial >> 32), bk, kStreamInit << 24));
        const uint64_t v0 = group_mask(2u * bk, m), v1 = group_mask(2u * bk + 1u, m);
        const uint64_t x1a = ((uint64_t)r.y << 32 | r.x) & v0, x1b = ((uint64_t)r.w << 32 | r.z) & v1;
        reinterpret_cast<uint4 *>(ring + s * WP)[bk] =
            make_uint4((uint32_t)x1a, (uint32_t)(x1a >> 32), (uint32_t)x1b, (uint32_t)(x1b >> 32));
      }
    }
    for (uint32_t s = 0; s < tb; ++s) {
      const uint32_t t = base + s * waves_total;
      if (t >= trial_count) break;
      const uint2 *Xr = random_init ? ring + s * WP : ring;
      for (uint32_t b = 0; b < NB; ++b) D[b * 64u + lane] = 0u;
      uint32_t R = 0, M = m_first;
      bool all_dec = false;
      uint64_t any0 = 0, any1 = 0;            // final round's x: some live node 0 / some 1
      for (uint32_t r = 1; r <= k_max; ++r) {
        bool done = true;
        // One round; ODD (M odd): no R-phase tie, so no "?" proposal and a
        // receiver's P-phase c0 = m - c1 -- only the p1 plane is staged and
        // counted (see p_phase_k).
        auto round = [&](auto odd_c, auto sure_c) {
          constexpr bool ODD = decltype(odd_c)::value;
          constexpr bool SURE = decltype(sure_c)::value;   // ODD and m > 2F: every receiver decides (decide_k)
          uint2 *P1 = reinterpret_cast<uint2 *>(P);   // ODD: x1-style p1 plane [XW] in P's space
          // ---- R-phase ("proposal phase", node.ts:46-82): c1 per receiver, c0 = M - c1
#pragma nounroll
          for (uint32_t b = 0; b < NB; ++b) {
            uint32_t a1[G];
            tally_groups_x1<G>(Xr, W, a1);
            if constexpr (ODD) {
              const uint32_t hi_t = M >> 1;
              uint32_t st = 0;
              Unroll<G>::run([&](auto gi) {
                constexpr int g = decltype(gi)::value;
                const uint64_t p1 = vcmp_gt(a1[g], hi_t + (uint32_t)g) & group_mask(b * G + g, m);   // node.ts:63-69
                st = writelane<2 * g>(st, (uint32_t)p1);
                st = writelane<2 * g + 1>(st, (uint32_t)(p1 >> 32));
              });
              if (lane < 2u * G) reinterpret_cast<uint32_t *>(P1 + b * G)[lane] = st;
            } else {
              const uint2 st = stage_proposals<false, G>(a1, b, m, M);
              if (lane < 4u * G) reinterpret_cast<uint32_t *>(P + b * G)[lane] = st.x;
              if constexpr (G > 16) {
                if (lane < 4u * G - 64u) reinterpret_cast<uint32_t *>(P + b * G)[64u + lane] = st.y;
              }
            }
          }
          if constexpr (ODD) {                         // padding group read by the pairwise tally
            if (lane < XW - NB * G) P1[NB * G + lane] = make_uint2(0u, 0u);
          }
          // ---- P-phase ("voting phase", node.ts:83-158)
          const uint32_t mF = m > F ? m - F : 0u;
          any0 = 0;
          any1 = 0;
#pragma nounroll
          for (uint32_t b = 0; b < NB; ++b) {
            uint32_t a0[G], a1[G];
            if constexpr (ODD) tally_groups_x1<G>(P1, W, a1);
            else tally_groups<G>(P, W, a0, a1);
            if constexpr (SURE && !STATE) {
              // Every live receiver decides this round, so the trial halts: no
              // x plane or decided bits are staged, only the outcome masks.
              Unroll<G>::run([&](auto gi) {
                constexpr int g = decltype(gi)::value;
                const uint64_t vm = group_mask(b * G + g, m);
                const uint64_t d0 = vcmp_lt(a1[g], mF + (uint32_t)g) & vm;   // node.ts:99
                any0 |= d0;
                any1 |= vm & ~d0;                                            // node.ts:102
                asm volatile("" : "+s"(any0), "+s"(any1));
              });
              continue;
            }
            uint32_t st = 0, dbb = D[b * 64u + lane];
            Unroll<G>::run([&](auto gi) {
              constexpr int g = decltype(gi)::value;
              const uint64_t vm = group_mask(b * G + g, m);
              const uint32_t Fg = F + (uint32_t)g;
              const uint64_t d0 = (ODD ? vcmp_lt(a1[g], mF + (uint32_t)g)   // c0 = m - c1 > F
                                       : vcmp_gt(a0[g], Fg)) & vm;          // node.ts:99
              const uint64_t d1 = (SURE ? vm : vcmp_gt(a1[g], Fg) & vm) & ~d0;   // node.ts:102
              const uint64_t rest = vm & ~(d0 | d1);
              uint64_t x1 = d1;
              if (rest) {
                const uint32_t a0g = ODD ? (m + 2u * (uint32_t)g) - a1[g] : a0[g];   // bias g
                const uint64_t ad1 = ballot_s(a1[g] > a0g) & rest;         // node.ts:108-109
                const uint64_t tie = ballot_s(a1[g] == a0g) & rest;        // node.ts:110-111
                x1 |= ad1;
                if (tie) {                                                // node.ts:111
                  const uint64_t trial = trial_id(keys, t);
                  x1 |= coin_ballot(keys, (uint32_t)trial, (uint32_t)(trial >> 32), b * G + g, r, tie);
                }
              }
              st = writelane<2 * g>(st, (uint32_t)x1);
              st = writelane<2 * g + 1>(st, (uint32_t)(x1 >> 32));
              dbb = select_lanes(dbb, dbb | (1u << g), d0 | d1);           // sticky decided bit (node.ts:100-105)
              any1 |= x1;
              any0 |= vm & ~x1;
              asm volatile("" : "+s"(any0), "+s"(any1));                   // fold per group
            });
            D[b * 64u + lane] = dbb;
            if (lane < 2u * G) reinterpret_cast<uint32_t *>(X + b * G)[lane] = st;
            // groups of this block that hold live receivers for this lane
            const uint32_t j0 = b * G;
            uint32_t expect = 0u;
            if (j0 + 1u < W) {
              const uint32_t nfull = (W - 1u - j0) < (uint32_t)G ? (W - 1u - j0) : (uint32_t)G;
              expect = nfull >= 32u ? ~0u : ((1u << nfull) - 1u);
            }
            if (W - 1u >= j0 && W - 1u < j0 + G && lane < tail_n) expect |= 1u << (W - 1u - j0);
            done = done && __all((dbb & expect) == expect);
          }
        };
        if (!(M & 1u)) round(std::false_type{}, std::false_type{});
        else if (m > 2u * F) round(std::true_type{}, std::true_type{});
        else round(std::true_type{}, std::false_type{});
        Xr = X;
        M = m;
        R = r;
        all_dec = done;
        if (all_dec) break;
      }
      // ---- outcome
      const uint32_t v = (any0 && any1) ? 2u : (any1 ? 1u : 0u);
      const uint32_t bin = all_dec ? (R * 3u + v) : v;
      if (bin < 64u) hc += (lane == bin) ? 1u : 0u;
      else if (lane == 0) atomicAdd(&lhist[bin], 1u);
      if (all_dec && v == 2u && lane == 0) atomicAdd(&lhist[hist_len - 1u], 1u);
      if constexpr (STATE) {
        if (lane == 0 && p.rounds_out) *p.rounds_out = all_dec ? R : 0u;
        if (p.node_out) {
          for (uint32_t c = lane; c < m; c += 64u) {
            const uint32_t j = c >> 6;
            const uint2 q = Xr[j];
            const uint64_t x1 = (uint64_t)q.y << 32 | q.x;
            bo_node_state ns;
            ns.killed = 0;
            ns.x = (int8_t)((x1 >> lane) & 1ull);
            ns.decided = (int8_t)((D[(j / G) * 64u + lane] >> (j % G)) & 1u);
            ns.pad = 0;
            ns.k = (int32_t)R + 1;
            p.node_out[p.live_ids[c]] = ns;
          }
        }
      }
    }
  }

  if (hc) atomicAdd(&lhist[lane], hc);
  __syncthreads();
  flush_hist(lhist, p);
}

template <int G>
hipError_t launch_b(const KParams &p, int grid, hipStream_t s) {
  if (p.node_out || p.rounds_out)
    hipLaunchKernelGGL((benor_lockstep_blocked_kernel<G, true>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  else
    hipLaunchKernelGGL((benor_lockstep_blocked_kernel<G, false>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  return hipGetLastError();
}

template hipError_t launch_b<11>(const KParams &, int, hipStream_t);
template hipError_t launch_b<12>(const KParams &, int, hipStream_t);
template hipError_t launch_b<13>(const KParams &, int, hipStream_t);
template hipError_t launch_b<14>(const KParams &, int, hipStream_t);
template hipError_t launch_b<15>(const KParams &, int, hipStream_t);
template hipError_t launch_b<16>(const KParams &, int, hipStream_t);
template hipError_t launch_b<17>(const KParams &, int, hipStream_t);
template hipError_t launch_b<18>(const KParams &, int, hipStream_t);
template hipError_t launch_b<19>(const KParams &, int, hipStream_t);
template hipError_t launch_b<20>(const KParams &, int, hipStream_t);
template hipError_t launch_b<21>(const KParams &, int, hipStream_t);
template hipError_t launch_b<22>(const KParams &, int, hipStream_t);

}  // namespace benor
