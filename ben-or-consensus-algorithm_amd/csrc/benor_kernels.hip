// benor_kernels.hip -- gfx950 (MI355X) kernels for the Ben-Or round loop.
//
// Replaces the reference's per-node POST /message handler
// (viviendbk/ben-or-consensus-algorithm src/nodes/node.ts:43-163) for a batch
// of independent trials.  Design:
//
//   * one wave64 = one trial (a whole simulated network), so the
//     all-to-all message exchange of a phase never leaves the wave: there are
//     no barriers, no inter-wave traffic and no HBM traffic in the round loop;
//   * lane l of receiver group j is live node c = 64 j + l (compact order of
//     live node ids); crashed nodes (node.ts:45,171) own no lane and no bit;
//   * a phase's messages are bit planes over the m live senders produced by
//     wave ballots (v_cmp -> SGPR lane mask): x planes carry is1 only (every
//     x is 0 or 1 after /start), proposal planes is0 and is1 ("?" is
//     neither) -- or is1 only when the vote count is odd and no "?" exists;
//   * every live receiver tallies its own inbox with v_bcnt_u32_b32
//     (popcount + accumulate, one VALU op per 32 senders per count), taking
//     each plane word as an SGPR straight from the ballot (W kernel) or from
//     a broadcast LDS read, and applying it to every receiver group of the lane;
//   * per-node coins (node.ts:111) and random initial values come from
//     Philox4x32-10 keyed by (seed, global trial id, node id, round);
//   * each trial's outcome is one increment of a per-wave counter, flushed to
//     HBM with one atomic per non-zero bin per workgroup.
//
// Per-receiver tallies are the simulated unit (SURVEY §7 "symmetry trap"):
// in lockstep mode all receivers of a trial see the same inbox, so a compiler
// would legitimately merge their identical popcounts.  The tally is therefore
// an opaque `v_bcnt_u32_b32` and each receiver group's chain starts from a
// distinct constant (subtracted afterwards) so that every live node's count is
// executed by its own lane, as the reference executes it in its own handler.
//
// This file: the random-delivery and event-level kernels, the popcount probe,
// and the host-side planning / dispatch.  The lockstep kernels live in
// benor_lane.h (m <= 64, one trial per lane), benor_w_kernel.h (W kernel,
// instantiated by benor_w_*.hip) and benor_blocked.hip (m > 2048).
#include <stdlib.h>

#include "benor_device.h"

#include <cstring>

namespace benor {

// ----------------------------------------- random-delivery kernel (f <= F)
// Generalised delivery: with f <= F crashed nodes every live
// receiver tallies, per phase, a uniformly random subset of exactly q = N-F of
// the m = N-f live senders ("first N-F arrivals"), drawn by Floyd's algorithm
// from Philox stream 2 (definition: oracle/benor_oracle.c
// oracle_delivery_mask).  The subset is built per lane in an LDS bitset laid
// out [word][lane] (any per-lane word index is bank-conflict free), then the
// receiver's inbox is (sender plane AND delivery mask).  One receiver group
// (64 receivers) at a time; this mode is bound by the subset's random draws.
// One Floyd step: sender t, else (t already in the subset) sender jj, joins
// the lane's bitset ([word][lane] in LDS, `lb` = this lane's byte offset).
// ds_or: LDS ops of a wave retire in order, so the next step's read sees this
// one.  Branch-free: idx = t + set * (jj - t) (t <= jj), and the shifts use the
// hardware's low-5-bit shift amounts.
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// LDS byte address of the bitset word holding `bit` for this lane:
// (bit >> 5) * 256 + lbase, lbase = the bitset's LDS address + lane * 4.
__device__ __forceinline__ lds_u32 *bitset_word(uint32_t bit, uint32_t lbase) {
  uint32_t a;                                          // v_lshrrev + v_lshl_add
  asm("v_lshl_add_u32 %0, %1, 8, %2" : "=v"(a) : "v"(bit >> 5), "v"(lbase));
  return (lds_u32 *)(uintptr_t)a;
}

__device__ __forceinline__ void floyd_insert(uint32_t lbase, uint32_t t, uint32_t jj) {
  const uint32_t cur = *bitset_word(t, lbase);
  const uint32_t set = __builtin_amdgcn_ubfe(cur, t, 1u);     // v_bfe_u32 reads offset bits [4:0]
  const uint32_t idx = t + __umul24(set, jj - t);
  __hip_atomic_fetch_or(bitset_word(idx, lbase), 1u << (idx & 31u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__device__ __forceinline__ void random_tally(const uint4 *__restrict__ plane, uint32_t *__restrict__ B,
                                             uint32_t W, uint32_t m, uint32_t q, bool active, uint32_t k0,
                                             uint32_t k1, uint32_t tlo, uint32_t thi, uint32_t node, uint32_t r,
                                             uint32_t phase, uint32_t &c0, uint32_t &c1) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t e = m - q;
  const bool deliver_T = q <= e;
  const uint32_t k = deliver_T ? q : e;
  // Floyd over [0, m): for jj = m-k .. m-1, t = uniform(jj + 1) (Lemire, exact).
  // Words come from Philox stream 2 in order (DStream above: word i is element
  // i & 3 of block i >> 2).  Fast path: one block = 4 draws, taken while the
  // lane's stream position is block-aligned and none of the 4 products needs
  // Lemire's exact rejection test; otherwise one exact DStream step (same
  // words, same result -- the oracle's definition).
  // delivery counter {tlo, thi, block | round << 16 | phase << 31, node | 2 << 24} (oracle_delivery_mask)
  const uint32_t c2 = ((r & 0x7FFFu) << 16) | ((phase & 1u) << 31), c3 = (node & 0xFFFu) | (kStreamDelivery << 24);
  const uint32_t lb = (uint32_t)(uintptr_t)(lds_u32 *)B + lane * 4u;   // LDS address of this lane's word 0
  uint32_t jj = m - k, widx = 0;
  for (;;) {
    const bool go = active && jj < m;
    if (!__any(go)) break;
    bool fast = go && (widx & 3u) == 0u;
    if (fast) {
      const uint4 b = philox4x32_10(k0, k1, make_uint4(tlo, thi, c2 | (widx >> 2), c3));
      const uint64_t q0 = (uint64_t)b.x * (jj + 1u), q1 = (uint64_t)b.y * (jj + 2u);
      const uint64_t q2 = (uint64_t)b.z * (jj + 3u), q3 = (uint64_t)b.w * (jj + 4u);
      // Lemire's exact test is needed only when a low word is below its range;
      // ranges grow with i, so one compare of the smallest low word against the
      // largest range is a safe screen (it may send a block to the exact path
      // needlessly, never the other way).
      const uint32_t lmin = min(min((uint32_t)q0, (uint32_t)q1), min((uint32_t)q2, (uint32_t)q3));
      if (lmin >= jj + 4u) {
        const uint32_t n = m - jj < 4u ? m - jj : 4u;          // draws left in this subset
        floyd_insert(lb, (uint32_t)(q0 >> 32), jj);
        if (n == 4u) {                                          // the common case: no per-step branch
          floyd_insert(lb, (uint32_t)(q1 >> 32), jj + 1u);
          floyd_insert(lb, (uint32_t)(q2 >> 32), jj + 2u);
          floyd_insert(lb, (uint32_t)(q3 >> 32), jj + 3u);
        } else {                                                // the subset's last block
          if (n > 1u) floyd_insert(lb, (uint32_t)(q1 >> 32), jj + 1u);
          if (n > 2u) floyd_insert(lb, (uint32_t)(q2 >> 32), jj + 2u);
        }
        jj += n;
        widx += n;
      } else {
        fast = false;
      }
    }
    if (go && !fast) {
      DStream ds;
      ds.k0 = k0; ds.k1 = k1; ds.c0 = tlo; ds.c1 = thi; ds.c2 = c2; ds.c3 = c3; ds.sh = 0u;
      ds.widx = widx & ~3u;                                      // refill the current block, then skip to widx
      for (uint32_t i = ds.widx; i < widx; ++i) (void)ds.next();
      const uint32_t t = ds.uniform(jj + 1u);
      floyd_insert(lb, t, jj);
      widx = ds.widx;
      ++jj;
    }
  }
  uint32_t a0 = 0, a1 = 0;
  for (uint32_t w = 0; w < W; ++w) {
    const uint4 rc = plane[w];
    const uint32_t tlo_w = B[(2u * w) * 64u + lane], thi_w = B[(2u * w + 1u) * 64u + lane];
    B[(2u * w) * 64u + lane] = 0u;
    B[(2u * w + 1u) * 64u + lane] = 0u;
    const uint64_t vm = group_mask(w, m);
    const uint32_t dlo = deliver_T ? tlo_w : ((uint32_t)vm & ~tlo_w);
    const uint32_t dhi = deliver_T ? thi_w : ((uint32_t)(vm >> 32) & ~thi_w);
    a0 += __builtin_popcount(rc.x & dlo) + __builtin_popcount(rc.y & dhi);
    a1 += __builtin_popcount(rc.z & dlo) + __builtin_popcount(rc.w & dhi);
  }
  c0 = a0;
  c1 = a1;
}

__global__ void __launch_bounds__(256) benor_random_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t m = p.m, F = p.F, W = p.W, q = p.q;

  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint4 *X = reinterpret_cast<uint4 *>(smem + p.hist_bytes + wv * p.wave_bytes);   // [W]
  uint4 *P = X + W;                                                                 // [W]
  uint32_t *B = reinterpret_cast<uint32_t *>(P + W);                                // [2W][64] bitset

  for (uint32_t i = threadIdx.x; i < p.hist_len; i += blockDim.x) lhist[i] = 0u;
  for (uint32_t w = 0; w < 2u * W; ++w) B[w * 64u + lane] = 0u;
  __syncthreads();

  uint64_t expect = 0ull;                          // groups holding a live receiver for this lane
  for (uint32_t j = 0; j < W; ++j)
    if (j * 64u + lane < m) expect |= 1ull << j;

  const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
  const uint64_t waves_total = (uint64_t)gridDim.x * kWavesPerBlock;

  for (uint64_t t = (uint64_t)blockIdx.x * kWavesPerBlock + wv; t < p.trial_count; t += waves_total) {
    const uint64_t trial = p.trial_begin + t;
    const uint32_t tlo = (uint32_t)trial, thi = (uint32_t)(trial >> 32);
    if (p.init_mode == BO_INIT_RANDOM) {           // /start (node.ts:167-188)
      const uint32_t nph = (W + 1u) >> 1;
      if (lane < nph) {
        uint4 r;
        if (m <= 32u) r = make_uint4(init_word_small(k0, k1, trial), 0u, 0u, 0u);   // shared block (m <= 32)
        else r = philox4x32_10(k0, k1, make_uint4(tlo, thi, lane, kStreamInit << 24));
        const uint32_t w0 = 2u * lane, w1 = w0 + 1u;
        const uint64_t v0 = group_mask(w0, m), v1 = group_mask(w1, m);
        const uint64_t x1a = ((uint64_t)r.y << 32 | r.x) & v0;
        X[w0] = rec(v0 & ~x1a, x1a);
        if (w1 < W) {
          const uint64_t x1b = ((uint64_t)r.w << 32 | r.z) & v1;
          X[w1] = rec(v1 & ~x1b, x1b);
        }
      }
    } else {
      for (uint32_t w = lane; w < W; w += 64u) X[w] = p.init_plane[w];
    }
    uint64_t dec = 0ull;
    uint32_t R = 0;
    bool all_dec = false;
    for (uint32_t r = 1; r <= p.k_max; ++r) {
      // ---- R-phase ("proposal phase", node.ts:46-82) over each receiver's first N-F arrivals
      for (uint32_t j = 0; j < W; ++j) {
        const uint32_t c = j * 64u + lane;
        const bool active = c < m;
        const uint32_t node = active ? p.live_ids[c] : 0u;
        uint32_t a0, a1;
        random_tally(X, B, W, m, q, active, k0, k1, tlo, thi, node, r, 0u, a0, a1);
        const uint64_t vm = group_mask(j, m);
        const uint64_t p0 = ballot(a0 > a1) & vm;
        const uint64_t p1 = ballot(a1 > a0) & vm;
        if (lane == 0) P[j] = rec(p0, p1);
      }
      // ---- P-phase ("voting phase", node.ts:83-158)
      for (uint32_t j = 0; j < W; ++j) {
        const uint32_t c = j * 64u + lane;
        const bool active = c < m;
        const uint32_t node = active ? p.live_ids[c] : 0u;
        uint32_t a0, a1;
        random_tally(P, B, W, m, q, active, k0, k1, tlo, thi, node, r, 1u, a0, a1);
        const uint64_t vm = group_mask(j, m);
        const bool d0l = a0 > F, d1l = a1 > F;
        const uint64_t d0 = ballot(d0l) & vm;
        const uint64_t d1 = ballot(d1l) & vm & ~d0;
        const uint64_t rest = vm & ~(d0 | d1);
        uint64_t x1 = d1;
        if (rest) {
          x1 |= ballot(a1 > a0) & rest;
          const uint64_t tie = ballot(a1 == a0) & rest;
          if (tie) x1 |= coin_ballot(k0, k1, tlo, thi, j, r, tie);
        }
        if (lane == 0) X[j] = rec(vm & ~x1, x1);
        if (d0l || d1l) dec |= 1ull << j;
      }
      R = r;
      all_dec = __all((dec & expect) == expect);
      if (all_dec) break;
    }
    bool any0 = false, any1 = false;
    if (lane < W) {
      const uint4 qq = X[lane];
      any0 = (qq.x | qq.y) != 0u;
      any1 = (qq.z | qq.w) != 0u;
    }
    const bool g0 = __any(any0), g1 = __any(any1);
    const uint32_t v = (g0 && g1) ? 2u : (g1 ? 1u : 0u);
    if (lane == 0) {
      atomicAdd(&lhist[all_dec ? (R * 3u + v) : v], 1u);
      if (all_dec && v == 2u) atomicAdd(&lhist[p.hist_len - 1u], 1u);
      if (p.rounds_out) *p.rounds_out = all_dec ? R : 0u;
    }
    if (p.node_out) {
      for (uint32_t c = lane; c < m; c += 64u) {
        const uint32_t j = c >> 6;
        const uint4 qq = X[j];
        const uint64_t x1 = (uint64_t)qq.w << 32 | qq.z;
        bo_node_state ns;
        ns.killed = 0;
        ns.x = (int8_t)((x1 >> lane) & 1ull);
        ns.decided = (int8_t)((dec >> j) & 1ull);
        ns.pad = 0;
        ns.k = (int32_t)R + 1;
        p.node_out[p.live_ids[c]] = ns;
      }
    }
  }

  __syncthreads();
  flush_hist(lhist, p);
}


// ------------------------------------------------ event-level kernel (N <= 256)
// message-granular simulation with the reference's literal
// handler (node.ts:45-158), a seeded delivery order and mid-run GET /stop
// (node.ts:191-194).  Definition: oracle/benor_oracle.c event_trial().  One
// lane = one trial; each lane runs its own event loop over a message pool in
// its slice of an HBM scratch buffer (pool of 4N^2+64 messages, per-node
// inbox counters for a 4-round window, x / k per node, completion masks,
// sorted crash list).  Exactly F nodes are crash-faulty from the start
// (launchNodes.ts:12-13), so every trigger fires once: the window of rounds a
// node can receive for is {k, k+1}, and round k's slots are recycled for
// round k+4.
__device__ __forceinline__ uint64_t splitmix64(uint64_t &s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Node-id bitsets of NW 64-bit words (N <= 64 NW; event mode N <= 256): a
// dynamic word index is resolved by selects over the NW registers.
template <int NW>
__device__ __forceinline__ bool set_has(const uint64_t (&m)[NW], uint32_t i) {
  uint64_t w = m[0];
#pragma unroll
  for (int j = 1; j < NW; ++j) w = (i >> 6) == (uint32_t)j ? m[j] : w;
  return (w >> (i & 63u)) & 1ull;
}
template <int NW>
__device__ __forceinline__ void set_add(uint64_t (&m)[NW], uint32_t i) {
  const uint64_t bit = 1ull << (i & 63u);
#pragma unroll
  for (int j = 0; j < NW; ++j) m[j] |= (i >> 6) == (uint32_t)j ? bit : 0ull;
}

// Messages are 16 bits: to | phase << 8 | x << 9 | (k & 3) << 11.  A message
// to a live receiver is for a round in [cur, cur + 2] (cur = the lowest round
// some running node has not completed: a receiver completes round k only
// after all m of its round-k messages arrived, and no node is more than one
// round ahead of cur), so k = cur + ((k - cur) & 3) recovers it; messages to
// killed receivers are dropped unread.  Half the pool bytes of a 32-bit form.
struct EvLane {
  uint16_t *pool;      // [cap] messages
  uint32_t *ibox;      // [N][4][2] packed {c0, c1, len}, 10 bits each
  uint64_t *comp;      // [4][NW] completion masks, round k at k & 3
  uint64_t *crash;     // [N] sorted (event << 8 | node)
  int8_t *xs;          // [N]
  int16_t *ks;         // [N]
};

// Inbox counters {c0, c1, len} of one (node, round slot, phase): in the lane's
// scratch slice as 10-bit fields of a u32, or -- LBOX, N <= kMaxEventLdsN -- in
// LDS as 5-bit fields of a u16, laid out [slot][lane of the workgroup].  The
// counter read-modify-write sits on every event's dependent path (its result
// decides the trigger, node.ts:52,88); in LDS it costs an LDS round trip
// instead of a second global-memory one.
template <bool LBOX>
struct EvBox {
  static constexpr uint32_t kSh = LBOX ? 5u : 10u;   // c0: bits 0.., c1: kSh.., len: 2 kSh..
  uint32_t *g;          // [N][4][2] (scratch)
  uint16_t *l;          // [N * 8][256] (LDS)
  uint32_t tid;
  __device__ __forceinline__ uint32_t get(uint32_t slot) const { return LBOX ? (uint32_t)l[slot * 256u + tid] : g[slot]; }
  __device__ __forceinline__ void set(uint32_t slot, uint32_t v) {
    if (LBOX) l[slot * 256u + tid] = (uint16_t)v;
    else g[slot] = v;
  }
};

template <int NW, bool LBOX>
__global__ void __launch_bounds__(256) benor_event_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  for (uint32_t i = threadIdx.x; i < p.hist_len; i += blockDim.x) lhist[i] = 0u;
  __syncthreads();

  const uint32_t N = p.N, F = p.F, quorum = p.N - p.F, m = p.m;
  uint64_t all[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    const uint32_t lo = 64u * (uint32_t)j;
    all[j] = N >= lo + 64u ? ~0ull : (N > lo ? (1ull << (N - lo)) - 1ull : 0ull);
  }
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
  const uint32_t cap = p.ev_cap;
  uint32_t *base = p.scratch + gid * p.ev_stride;
  EvLane L;
  L.pool = reinterpret_cast<uint16_t *>(base);
  L.ibox = base + (((cap + 1u) >> 1) + 1u & ~1u);     // pool words, even (comp is 8-byte aligned)
  L.comp = reinterpret_cast<uint64_t *>(L.ibox + N * 8u);
  L.crash = L.comp + 4 * NW;
  L.xs = reinterpret_cast<int8_t *>(L.crash + N);
  L.ks = reinterpret_cast<int16_t *>(L.xs + ((N + 3u) & ~3u));
  EvBox<LBOX> box;
  box.g = L.ibox;
  box.l = reinterpret_cast<uint16_t *>(smem + p.hist_bytes);
  box.tid = threadIdx.x;
  constexpr uint32_t kSh = EvBox<LBOX>::kSh, kMask = (1u << kSh) - 1u;
  const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);

  auto full = [&](const uint64_t *a, const uint64_t (&b)[NW]) {   // a | b == all
    bool f = true;
#pragma unroll
    for (int j = 0; j < NW; ++j) f = f && (a[j] | b[j]) == all[j];
    return f;
  };

  for (uint64_t t = gid; t < p.trial_count; t += lanes) {
    const uint64_t trial = p.trial_begin + t;
    const uint32_t tlo = (uint32_t)trial, thi = (uint32_t)(trial >> 32);
    uint64_t killed[NW], decided[NW];
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      killed[j] = p.faulty_mask[j];
      decided[j] = 0ull;
    }
    // ---- node.ts:21-26 and initial values (compact live order): word c >> 5 of stream 1
    uint4 ir = make_uint4(0, 0, 0, 0);
    for (uint32_t c = 0; c < m; ++c) {
      const uint32_t i = p.live_ids[c];
      int8_t v;
      if (p.init_mode == BO_INIT_RANDOM) {
        if (m <= 32u) {                              // the shared block of four trials (oracle_random_init)
          if (c == 0u) ir = init_block_small(k0, k1, trial >> 2);
          const uint32_t w = coin_word_v(ir, (uint32_t)(trial & 3u) + 1u);
          v = (int8_t)((w >> c) & 1u);
        } else {
          if ((c & 127u) == 0u) ir = philox4x32_10<false>(k0, k1, make_uint4(tlo, thi, c >> 7, kStreamInit << 24));
          const uint32_t j = (c >> 5) & 3u;
          const uint32_t w = j == 0u ? ir.x : j == 1u ? ir.y : j == 2u ? ir.z : ir.w;
          v = (int8_t)((w >> (c & 31u)) & 1u);
        }
      } else {
        v = p.init_x[i];
      }
      L.xs[i] = v;
      L.ks[i] = 0;
    }
    for (uint32_t i = 0; i < N; ++i)
      if (set_has(killed, i)) { L.xs[i] = -1; L.ks[i] = -1; }
    for (uint32_t j = 0; j < N * 8u; ++j) box.set(j, 0u);
    for (int j = 0; j < 4 * NW; ++j) L.comp[j] = 0ull;
    // ---- mid-run /stop schedule, sorted by event index
    uint32_t ncrash = 0;
    if (p.crash_at) {
      for (uint32_t i = 0; i < N; ++i)
        if (p.crash_at[i] != 0xFFFFFFFFu) L.crash[ncrash++] = ((uint64_t)p.crash_at[i] << 8) | i;
    } else if (p.crash_count > 0 && m > 0 && p.crash_window > 0) {
      DStream ds;
      ds.k0 = k0; ds.k1 = k1; ds.c0 = tlo; ds.c1 = thi; ds.c2 = 0u; ds.c3 = kStreamCrash << 24; ds.widx = 0;
      ds.sh = 12u;
      const uint32_t kk = p.crash_count < m ? p.crash_count : m;
      // Floyd over compact live indices; the picks go to the crash list first
      // (node field = compact index), then get their event indices in pick order
      uint64_t T[NW];
#pragma unroll
      for (int j = 0; j < NW; ++j) T[j] = 0ull;
      for (uint32_t j = m - kk; j < m; ++j) {
        const uint32_t tt = ds.uniform(j + 1u);
        const uint32_t idx = set_has(T, tt) ? j : tt;
        set_add(T, idx);
        L.crash[ncrash++] = idx;
      }
      for (uint32_t q2 = 0; q2 < kk; ++q2) {
        const uint32_t when = ds.uniform(p.crash_window);
        L.crash[q2] = ((uint64_t)when << 8) | p.live_ids[(uint32_t)L.crash[q2]];
      }
    }
    for (uint32_t a = 1; a < ncrash; ++a) {            // insertion sort (<= N entries)
      const uint64_t v = L.crash[a];
      uint32_t b = a;
      while (b > 0 && L.crash[b - 1] > v) { L.crash[b] = L.crash[b - 1]; --b; }
      L.crash[b] = v;
    }
    uint32_t next = 0;
    // ---- delivery order
    uint64_t rng;
    {
      const uint4 o = philox4x32_10<false>(k0, k1, make_uint4(tlo, thi, 0u, kStreamOrder << 24));
      rng = (((uint64_t)o.x << 32) | o.y) ^ 0xD1B54A32D192ED03ull;
    }
    // ---- /start (node.ts:167-188)
    uint32_t len = 0;
    for (uint32_t i = 0; i < N; ++i) {
      if (set_has(killed, i)) continue;
      L.ks[i] = 1;
      const uint32_t body = ((uint32_t)(L.xs[i] & 3) << 9) | (1u << 11);
      for (uint32_t to = 0; to < N; ++to) L.pool[len++] = (uint16_t)(to | body);
    }
    uint32_t cur = 1, R = 0, halted = 0;
    bool overflow = false;
    for (uint64_t e = 0;; ++e) {
      // scheduled GET /stop (node.ts:191-194)
      bool crashed = false;
      while (next < ncrash && (L.crash[next] >> 8) == e) {
        set_add(killed, (uint32_t)(L.crash[next] & 255u));
        crashed = true;
        ++next;
      }
      if (crashed) {
        bool dead = true;
#pragma unroll
        for (int j = 0; j < NW; ++j) dead = dead && killed[j] == all[j];
        if (dead) { halted = 3; break; }
        while (full(L.comp + (cur & 3u) * NW, killed)) {
          if (full(decided, killed)) { halted = 1; R = cur; break; }
          if (cur >= p.k_max) { halted = 2; R = cur; break; }
          for (int j = 0; j < NW; ++j) L.comp[(cur & 3u) * NW + j] = 0ull;
          ++cur;
        }
        if (halted) break;
      }
      if (len == 0) { halted = 3; break; }
      const uint32_t pick = (uint32_t)(((uint64_t)(uint32_t)(splitmix64(rng) >> 32) * (uint64_t)len) >> 32);
      const uint32_t msg = L.pool[pick];
      L.pool[pick] = L.pool[--len];
      const uint32_t to = msg & 255u, ph = (msg >> 8) & 1u, k = cur + (((msg >> 11) - cur) & 3u);
      const uint32_t x = (msg >> 9) & 3u;
      if (set_has(killed, to)) continue;               // node.ts:45
      const uint32_t slot = (to * 4u + (k & 3u)) * 2u + ph;
      uint32_t b = box.get(slot);
      b += 1u << (2u * kSh);                           // len
      if (x == 0u) b += 1u;                            // c0
      else if (x == 1u) b += 1u << kSh;                // c1
      box.set(slot, b);
      if ((b >> (2u * kSh)) != quorum) continue;       // node.ts:52, :88 (fires once: exactly F faulty)
      const uint32_t c0 = b & kMask, c1 = (b >> kSh) & kMask;
      uint32_t body;
      if (ph == 0u) {                                  // node.ts:53-80
        const uint32_t v = c0 > c1 ? 0u : (c1 > c0 ? 1u : 2u);
        body = (1u << 8) | (v << 9) | ((k & 3u) << 11);
      } else {                                         // node.ts:89-157
        int8_t nx;
        if (c0 > F) { nx = 0; set_add(decided, to); }
        else if (c1 > F) { nx = 1; set_add(decided, to); }
        else if (c0 + c1 > 0 && c0 > c1) nx = 0;
        else if (c0 + c1 > 0 && c0 < c1) nx = 1;
        else {
          // compact index of `to` (coin_block, node.ts:111)
          uint32_t c = 0;
#pragma unroll
          for (int j = 0; j < NW; ++j) {
            const uint32_t lo = 64u * (uint32_t)j;
            const uint64_t below = to >= lo + 64u ? ~0ull : (to > lo ? (1ull << (to - lo)) - 1ull : 0ull);
            c += (uint32_t)__builtin_popcountll(~p.faulty_mask[j] & below & all[j]);
          }
          const uint4 rr = philox4x32_10<false>(k0, k1, make_uint4(tlo, thi, c >> 5, ((k - 1u) >> 2) | (kStreamCoin << 24)));
          nx = (int8_t)((coin_word_v(rr, k) >> (c & 31u)) & 1u);
        }
        L.xs[to] = nx;
        L.ks[to] = (int16_t)(k + 1u);
        box.set((to * 4u + ((k + 2u) & 3u)) * 2u + 0u, 0u);   // recycle round k-2's slots for k+2
        box.set((to * 4u + ((k + 2u) & 3u)) * 2u + 1u, 0u);
        L.comp[(k & 3u) * NW + (to >> 6)] |= 1ull << (to & 63u);
        while (full(L.comp + (cur & 3u) * NW, killed)) {
          if (full(decided, killed)) { halted = 1; R = cur; break; }
          if (cur >= p.k_max) { halted = 2; R = cur; break; }
          for (int j = 0; j < NW; ++j) L.comp[(cur & 3u) * NW + j] = 0ull;
          ++cur;
        }
        if (halted) break;
        body = ((uint32_t)(nx & 3) << 9) | (((k + 1u) & 3u) << 11);
      }
      if (len + N > cap) { overflow = true; halted = 3; break; }
      for (uint32_t dst = 0; dst < N; ++dst) L.pool[len++] = (uint16_t)(dst | body);
    }
    // ---- outcome over the nodes still running
    bool any0 = false, any1 = false, anyq = false;
    uint32_t nlive = 0;
    for (uint32_t i = 0; i < N; ++i) {
      if (set_has(killed, i)) continue;
      ++nlive;
      const int8_t v = L.xs[i];
      if (v == 0) any0 = true; else if (v == 1) any1 = true; else anyq = true;
    }
    const uint32_t v = (nlive == 0 || anyq || (any0 && any1)) ? 2u : (any1 ? 1u : 0u);
    atomicAdd(&lhist[halted == 1 ? (R * 3u + v) : v], 1u);
    if (halted == 1 && v == 2u) atomicAdd(&lhist[p.hist_len - 1u], 1u);
    if (overflow && p.rounds_out) atomicOr(p.rounds_out, 0x80000000u);
    if (overflow && p.overflow) atomicOr(p.overflow, 2u);   // bo_plan_check: the pool filled up
    if (p.node_out) {
      for (uint32_t i = 0; i < N; ++i) {
        const bool f = (p.faulty_mask[i >> 6] >> (i & 63u)) & 1ull;
        bo_node_state ns;
        ns.killed = (int8_t)(set_has(killed, i) ? 1 : 0);
        ns.x = L.xs[i];
        ns.decided = f ? (int8_t)-1 : (int8_t)(set_has(decided, i) ? 1 : 0);
        ns.pad = 0;
        ns.k = L.ks[i];
        p.node_out[i] = ns;
      }
      if (p.rounds_out) atomicOr(p.rounds_out, halted == 1 ? R : 0u);
    }
  }

  __syncthreads();
  flush_hist(lhist, p);
}

// --------------------------------------------------- popcount peak probe
// Eight independent v_bcnt_u32_b32 chains per lane; the roofline's `peak`
// is the spec VALU rate, this probe says what the part sustains.
__global__ void __launch_bounds__(256) popc_peak_kernel(uint32_t *sink, int iters) {
  uint32_t a[8];
  const uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = x + (uint32_t)i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(a[i]) : "v"(x));
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= a[i];
  if (s == 0x12345678u) sink[blockIdx.x] = s;
}

// ------------------------------------------------------------ host side
void plan_geometry(KParams &p) {
  const uint32_t W = p.W;
  p.hist_len = (p.k_max + 1u) * 3u + 1u;
  p.hist_bytes = (((p.hist_len * 4u) + 15u) & ~15u) + kParamBytes;   // histogram + parameter block
  // one wave per trial (benor_event_big.hip), or one workgroup per trial
  // (benor_event_live.hip: live runs; batch plans under BENOR_EVENT_FORM=wg or wave)
  const bool wg = p.mode == BO_MODE_EVENT &&
                  (p.live || knob_is("BENOR_EVENT_FORM", "wg") || knob_is("BENOR_EVENT_FORM", "wave"));
  if (p.mode == BO_MODE_EVENT && (p.N > kMaxEventN || wg)) {
    p.G = 1;
    p.nblocks = 1;
    p.variant = 5;
    p.wave_bytes = 0;
    p.ev_wg = wg ? 1u : 0u;
    p.ev_cap = 4u * p.N * p.N + 64u;
    p.ev_stride = p.ev_cap;                          // u32 messages
    p.lds_bytes = wg ? event_wg_lds_bytes(p, event_wg_waves(p)) : event_big_lds_bytes(p);
    return;
  }
  if (p.mode == BO_MODE_EVENT) {
    p.G = 1;
    p.nblocks = 1;
    p.variant = 4;
    p.wave_bytes = 0;
    // N <= kMaxEventLdsN: the inbox counters live in LDS, 8N u16 per lane of the
    // 256-lane workgroup (EvBox)
    p.lds_bytes = p.hist_bytes + (p.N <= kMaxEventLdsN ? 256u * 8u * p.N * 2u : 0u);
    const uint32_t NW = p.N <= 64u ? 1u : 4u;
    p.ev_cap = 4u * p.N * p.N + 64u;
    // per-lane scratch (u32 words): pool, inbox window, comp[4][NW] (u64), crash[N] (u64), xs (i8), ks (i16)
    p.ev_stride = (((p.ev_cap + 1u) >> 1) + 1u & ~1u) + p.N * 8u + 8u * NW + 2u * p.N + ((p.N + 3u) & ~3u) / 4u +
                  (p.N + 1u) / 2u;
    p.ev_stride = (p.ev_stride + 31u) & ~31u;
    return;
  }
  if (p.mode == BO_MODE_RANDOM_DELIVERY) {
    p.G = 1;
    p.nblocks = W;
    p.variant = 2;
    // sampler choice and parameters: oracle_delivery_bernoulli
    const uint32_t e = p.m - p.q, k = p.q <= e ? p.q : e;
    p.rd_a = p.rd_b = 0u;
    if (k >= 64u && (uint64_t)k * 8u > p.m) {
      uint32_t a = (16u * p.q + p.m - 1u) / p.m;
      p.rd_a = a < 1u ? 1u : (a > 15u ? 15u : a);
      uint32_t b = 1u;
      while ((1u << b) < p.m) ++b;
      p.rd_b = b;
    }
    p.wave_bytes = 2u * W * 16u + 2u * W * 64u * 4u;   // X, P records + per-lane bitset (Floyd)
    if (p.rd_a) {                                     // Bernoulli sampler (benor_random.hip): padded bitset rows
      p.rd_rows = random_bern_rows(p.m, p.rd_b);
      p.wave_bytes = 2u * W * 16u + p.rd_rows * 64u * 4u;
    }
    p.lds_bytes = p.hist_bytes + kWavesPerBlock * p.wave_bytes;
    return;
  }
  if (p.m <= kMaxLaneM) {                           // lane kernel: one trial per lane
    const uint32_t M1 = p.m - p.init_q;
    const bool odd = (p.m & 1u) && (M1 & 1u);        // every vote count odd: no tie, no coin
    p.G = odd ? (p.m > 2u * p.F ? 2u : 1u) : 0u;     // KIND (benor_lane.hip)
    p.nblocks = 1;
    p.variant = 6;
    p.wave_bytes = 128u * 8u + 128u * 16u;          // init-word ring, coin-block ring
    p.lds_bytes = p.hist_bytes + kWavesPerBlock * p.wave_bytes;
    // Packed matrix-core kernel (benor_mfma_small.h): 2 <= m <= 32, every
    // trial can decide (m > F) and no "?" initial value (every vote count is
    // m).  The lane kernel planned above serves the state launches (network
    // API); the packed kernel re-runs its rare leftovers itself.
    if (p.m >= 2u && p.m <= kMaxSmallMfmaM && p.m > p.F && p.init_q == 0u && !knob_is("BENOR_NO_MFMA", "1")) {
      p.base_variant = p.variant;
      p.base_G = p.G;
      p.variant = 8;
      p.lds_bytes = p.hist_bytes + kWavesPerBlock * small_wave_words(p.m) * 4u;   // histogram, round lists
    }
    return;
  }
  const uint32_t nph = (W + 1u) / 2u, tb = 64u / nph;   // init ring: tb trials per Philox pass
  const uint32_t WP = 2u * nph;                         // x1 words per plane row (even)
  if (W <= (uint32_t)kMaxWSpecialised) {
    p.G = W;
    p.nblocks = 1;
    p.variant = 1;
    p.wave_bytes = (tb * WP + 2u * WP) * 8u;            // init ring, final x1 plane, decided bits
  } else {
    // Blocks of G = ceil(W / nb) in 11..22 groups: the fewest padded groups nb * G,
    // ties to fewer blocks (larger G: more v_bcnt per LDS read and loop step, which
    // outweighs 4-5 waves/SIMD at G > 16 against 5-7 at G <= 16).  v19 A/B
    // (profiles/r01-v19_ab_blocked_g.txt): one padded group fewer is +3-7 %; on ties
    // the larger G is -0.3..+1.9 %.
    uint32_t nb = (W + 15u) / 16u, G = (W + nb - 1u) / nb;
    for (uint32_t n = (W + 21u) / 22u; n <= (W + 10u) / 11u; ++n) {
      const uint32_t g = (W + n - 1u) / n;
      if (g < 11u || g > 22u) continue;
      const bool better = n * g < nb * G || (n * g == nb * G && n < nb);
      if (better) {
        nb = n;
        G = g;
      }
    }
    const uint32_t XW = ((G * nb > WP ? G * nb : WP) + 1u) & ~1u;
    p.G = G;
    p.nblocks = nb;
    p.variant = 0;
    p.wave_bytes = (tb * WP + XW) * 8u + G * nb * 16u + nb * 256u;   // ring, x1 plane, {p0,p1} plane, decided bits
  }
  // Matrix-core kernel (benor_mfma.h) for round 1 wherever a trial can halt
  // there (m > F; not a fixed start whose round 1 ties for every trial).
  // KIND 0: all vote counts odd (m odd, even number of "?") and m > 2F --
  // every trial halts in round 1; KIND 1: m > 2F; KIND 2: F < m <= 2F.
  // Trials that do not halt in round 1 go to the popcount kernel planned
  // above (trial-list mode), as do the state launches (network API), so its
  // LDS plan stays.
  const bool sure = (p.m & 1u) && !(p.init_q & 1u) && p.m > 2u * p.F;
  const bool can_halt = p.m > p.F && !(p.init_mode == BO_INIT_FIXED && p.init_tie);
  const bool big_ok = !knob_is("BENOR_NO_MFMA_BIG", "1");
  if (can_halt && (p.m <= kMaxMfmaM || big_ok) && !knob_is("BENOR_NO_MFMA", "1")) {
    p.base_variant = p.variant;
    p.base_G = p.G;
    p.variant = 7;
    p.G = sure ? 0u : (p.m > 2u * p.F ? 1u : 2u);
  }
  p.lds_bytes = p.hist_bytes + kWavesPerBlock * p.wave_bytes;
}

template <int... Is>
static hipError_t dispatch_w(const KParams &p, int grid, hipStream_t s, std::integer_sequence<int, Is...>) {
  hipError_t e = hipErrorInvalidValue;
  (void)((p.W == (uint32_t)(Is + 2) ? (e = launch_w<Is + 2>(p, grid, s), true) : false) || ...);
  return e;
}

template <int... Is>
static hipError_t dispatch_lane(const KParams &p, int grid, hipStream_t s, std::integer_sequence<int, Is...>) {
  hipError_t e = hipErrorInvalidValue;
  (void)((p.m == (uint32_t)(Is + 1) ? (e = launch_lane_m<Is + 1>(p, grid, s), true) : false) || ...);
  return e;
}

template <int... Is>
static hipError_t dispatch_mfma_small(const KParams &p, int grid, hipStream_t s, std::integer_sequence<int, Is...>) {
  hipError_t e = hipErrorInvalidValue;
  (void)((p.m == (uint32_t)(Is + 2) ? (e = launch_mfma_small_m<Is + 2>(p, grid, s), true) : false) || ...);
  return e;
}

template <int... Is>
static hipError_t dispatch_mfma(const KParams &p, int grid, hipStream_t s, std::integer_sequence<int, Is...>) {
  hipError_t e = hipErrorInvalidValue;
  (void)((p.W == (uint32_t)(Is + 2) ? (e = launch_mfma<Is + 2>(p, grid, s), true) : false) || ...);
  return e;
}

// W in 33..64: G in 11..22 (plan_geometry)
template <int... Is>
static hipError_t dispatch_b(const KParams &p, int grid, hipStream_t s, std::integer_sequence<int, Is...>) {
  hipError_t e = hipErrorInvalidValue;
  (void)((p.G == (uint32_t)(Is + 11) ? (e = launch_b<Is + 11>(p, grid, s), true) : false) || ...);
  return e;
}

hipError_t launch_lockstep(const KParams &p, int grid, hipStream_t s) {
  if (p.variant == 4) {
    if (p.N <= kMaxEventLdsN) {
      if (p.lds_bytes > 64u * 1024u) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&benor_event_kernel<1, true>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds_bytes);
        if (e != hipSuccess) return e;
      }
      hipLaunchKernelGGL((benor_event_kernel<1, true>), dim3(grid), dim3(256), p.lds_bytes, s, p);
    } else if (p.N <= 64u) {
      hipLaunchKernelGGL((benor_event_kernel<1, false>), dim3(grid), dim3(256), p.lds_bytes, s, p);
    } else {
      hipLaunchKernelGGL((benor_event_kernel<4, false>), dim3(grid), dim3(256), p.lds_bytes, s, p);
    }
    return hipGetLastError();
  }
  if (p.variant == 5) return p.ev_wg ? launch_event_wg(p, grid, s) : launch_event_big(p, grid, s);
  if (p.variant == 6) return dispatch_lane(p, grid, s, std::make_integer_sequence<int, (int)kMaxLaneM>{});
  if (p.variant == 8 && !small_on_lane(p))
    return dispatch_mfma_small(p, grid, s, std::make_integer_sequence<int, (int)kMaxSmallMfmaM - 1>{});   // m = 2..32
  if (p.variant == 8) {                      // state launch or short launch of a packed shape: the lane kernel
    KParams q = p;
    q.variant = p.base_variant;
    q.G = p.base_G;
    q.lds_bytes = q.hist_bytes + kWavesPerBlock * q.wave_bytes;
    return launch_lockstep(q, grid, s);
  }
  if (p.variant == 2 && p.rd_a) return launch_random_bern(p, grid, s);
  if (p.variant == 2) {                      // Floyd sampler
    if (p.lds_bytes > 64u * 1024u) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&benor_random_kernel),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds_bytes);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(benor_random_kernel, dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
    return hipGetLastError();
  }
  if (p.variant == 7 && !p.node_out && !p.rounds_out) {
    if (p.W > 16u) return launch_mfma_big(p, grid, s);                                                        // W = 17..64
    return dispatch_mfma(p, grid, s, std::make_integer_sequence<int, 15>{});                                  // W = 2..16
  }
  if (p.variant == 7) {                      // state launch of a matrix-core shape: its popcount kernel
    KParams q = p;
    q.variant = p.base_variant;
    q.G = p.base_G;
    return launch_lockstep(q, grid, s);
  }
  if (p.variant == 1)
    return dispatch_w(p, grid, s, std::make_integer_sequence<int, kMaxWSpecialised - 1>{});                    // W = 2..32
  return dispatch_b(p, grid, s, std::make_integer_sequence<int, 12>{});
}

// The big-network matrix-core kernel holds 9-33 KB of LDS per wave; its
// workgroup size is chosen for occupancy (mfma_big_block_waves).  Every other
// kernel: kWavesPerBlock.
uint32_t block_waves(const KParams &p) {
  if (mfma_big_coop(p)) return mfma_coop_block_waves(p);
  return (p.variant == 7 && p.W > 16u && !p.node_out && !p.rounds_out) ? mfma_big_block_waves(p) : (uint32_t)kWavesPerBlock;
}

uint64_t defer_units(const KParams &p, int grid) {
  return mfma_big_coop(p) ? (uint64_t)grid : (uint64_t)grid * block_waves(p);
}

// A packed-shape launch runs on the lane kernel when it writes per-node
// state (network API) or is short: below ~10^6 trials the packed kernel's
// partial round lists at the end of each wave outweigh its per-trial gain
// (DESIGN §4.2).
// BENOR_SMALL_MIN_TRIALS overrides the crossover (validation knob).
bool small_on_lane(const KParams &p) {
  if (p.node_out || p.rounds_out) return true;
  return p.trial_count < knob_u32("BENOR_SMALL_MIN_TRIALS", (uint32_t)kSmallMinTrials);
}

int lockstep_grid(const KParams &p, int device) {
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (p.variant == 5) {   // big event level: one wave per trial, grid = the scratch's trial slots
    const uint64_t g = p.trial_count < p.ev_lanes ? p.trial_count : p.ev_lanes;
    return (int)(g < 1u ? 1u : g);
  }
  if (p.variant == 4) {   // event mode: one lane per trial, grid = the scratch's lane count
    const uint64_t blocks_needed = (p.trial_count + 255u) / 256u;
    uint64_t grid = p.ev_lanes / 256u;
    if (blocks_needed < grid) grid = blocks_needed;
    return (int)(grid < 1 ? 1 : grid);
  }
  if (p.variant == 8) {
    if (small_on_lane(p)) {                  // state launch or short launch: the lane kernel
      KParams q = p;
      q.variant = p.base_variant;
      q.G = p.base_G;
      q.lds_bytes = q.hist_bytes + kWavesPerBlock * q.wave_bytes;
      return lockstep_grid(q, device);
    }
    // Packed matrix-core kernel: a wave runs batches of 64 S trials (fresh
    // round-1 batches strided over the waves, then its own round lists), so
    // each wave gets ~3 fresh batches, at most 4 workgroups per CU.
    const uint64_t batch = 64u * small_slots(p.m);
    const uint64_t groups = (p.trial_count + batch - 1u) / batch;
    uint64_t per_cu = groups / ((uint64_t)cus * kWavesPerBlock * 3u);
    uint64_t cap = lds_groups_per_cu(p.lds_bytes);
    if (cap > 4u) cap = 4u;
    if (per_cu > cap) per_cu = cap;
    if (per_cu < 1u) per_cu = 1u;
    {                                        // tuning knob
      const uint64_t v = knob_u32("BENOR_BLOCKS_PER_CU", 0u);
      if (v >= 1u && v <= lds_groups_per_cu(p.lds_bytes)) per_cu = v;
    }
    uint64_t grid = (uint64_t)cus * per_cu;
    const uint64_t need = (groups + kWavesPerBlock - 1u) / kWavesPerBlock;
    if (need < grid) grid = need;
    return (int)(grid < 1u ? 1u : grid);
  }
  if (mfma_big_coop(p)) {   // cooperative big-network form: one 32-trial group per workgroup at a time
    const uint64_t groups = (p.trial_count + 31u) / 32u;
    uint64_t grid = (uint64_t)cus * (uint64_t)mfma_coop_blocks_per_cu(p);
    if (groups < grid) grid = groups;
    return (int)(grid < 1u ? 1u : grid);
  }
  // 32 waves per CU when registers and LDS allow it.
  const bool mfma = p.variant == 7 && !p.node_out && !p.rounds_out;
  const uint64_t per_wave = p.variant == 6 ? 64u : (mfma ? 32u : 1u);   // trials a wave runs at once
  const uint64_t waves_needed = (p.trial_count + per_wave - 1u) / per_wave;
  const uint32_t bw = block_waves(p);
  const uint64_t blocks_needed = (waves_needed + bw - 1) / bw;
  uint64_t per_cu = 32u / bw;
  // the matrix-core kernel uses no wave slices (its big-network form: proposal planes)
  const uint32_t lds = mfma ? (p.W > 16u ? mfma_big_lds_bytes(p, bw) : p.hist_bytes) : p.lds_bytes;
  if (lds > 0) {
    const uint64_t lds_fit = lds_groups_per_cu(lds);
    if (lds_fit < per_cu) per_cu = lds_fit ? lds_fit : 1;
  }
  // Lane kernel: a short launch spread over every wave slot (~2 trials per
  // lane at 10^6 trials) spends most of its time in per-wave overhead (ring
  // fills, the LDS histogram) and, with coin rounds (KIND 0), in the tail of
  // each wave's slowest trial.  Fewer, longer-lived waves: at least ~8
  // trial-rounds of work per lane, 2..8 workgroups per CU
  // (tools/lane_grid_sweep.py, profiles/r02_lane_grid.jsonl: N=10 F=4 at
  // 10^6 trials 41-57 us at 8 per CU, 22.5 us at 2; N=64 F=21 (KIND 2) 28.9 ->
  // 18.6 us; N=10 F=5 (KIND 1, k_max rounds per trial) keeps 8; at 10^7
  // trials 8 per CU stays best).
  if (p.variant == 6) {
    const uint64_t rounds = p.G == 1u ? (p.m <= p.F ? p.k_max : 2u) : 1u;   // per trial, roughly
    const uint64_t want = p.trial_count * rounds / ((uint64_t)cus * 64u * kWavesPerBlock * 8u);
    const uint64_t v = want < 2u ? 2u : want;
    if (v < per_cu) per_cu = v;
  }
  {                                          // tuning knob (tools/lane_grid_sweep.py)
    const uint64_t v = knob_u32("BENOR_BLOCKS_PER_CU", 0u);
    if (v >= 1u && v < per_cu) per_cu = v;
  }
  uint64_t grid = (uint64_t)cus * per_cu;
  if (blocks_needed < grid) grid = blocks_needed;
  if (grid < 1) grid = 1;
  return (int)grid;
}

hipError_t launch_popc_peak(uint32_t *sink, int grid, int iters, hipStream_t s, double *words) {
  hipLaunchKernelGGL(popc_peak_kernel, dim3(grid), dim3(256), 0, s, sink, iters);
  if (words) *words = (double)grid * 256.0 * (double)iters * 64.0;
  return hipGetLastError();
}

}  // namespace benor
