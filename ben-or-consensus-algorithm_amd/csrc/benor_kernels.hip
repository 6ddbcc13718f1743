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
//   * a phase's messages are two bit planes over the m live senders,
//     {is0, is1}, produced by wave ballots and kept in the wave's LDS slice as
//     16-byte records {is0.lo, is0.hi, is1.lo, is1.hi} per 64 senders;
//   * every live receiver tallies its own inbox with v_bcnt_u32_b32
//     (popcount + accumulate, one VALU op per 32 senders per count), reading
//     each record once per wave with a broadcast ds_read_b128 and applying it
//     to G receiver groups per lane;
//   * per-node coins (node.ts:111) and random initial values come from
//     Philox4x32-10 keyed by (seed, global trial id, node id, round);
//   * each trial's outcome is one increment of an LDS histogram, flushed to
//     HBM with one atomic per non-zero bin per workgroup.
//
// Per-receiver tallies are the simulated unit (SURVEY §7 "symmetry trap"):
// in lockstep mode all receivers of a trial see the same inbox, so a compiler
// would legitimately merge their identical popcounts.  The tally is therefore
// an opaque `v_bcnt_u32_b32` and each receiver group's chain starts from a
// distinct constant (subtracted afterwards) so that every live node's count is
// executed by its own lane, as the reference executes it in its own handler.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "benor_internal.h"

#ifndef BENOR_FUSED
#define BENOR_FUSED 1
#endif

namespace benor {

// ------------------------------------------------------------------ Philox
__device__ __forceinline__ uint4 philox4x32_10(uint32_t k0, uint32_t k1, uint4 c) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x;
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// One receiver's tally step: acc + popcount(word).  Opaque on purpose (see
// the header comment): the per-receiver count must execute per receiver.
__device__ __forceinline__ uint32_t tally(uint32_t word, uint32_t acc) {
  uint32_t r;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(word), "v"(acc));
  return r;
}

__device__ __forceinline__ uint64_t group_mask(uint32_t j, uint32_t m) {
  const uint32_t lo = j * 64u;
  if (lo >= m) return 0ull;
  const uint32_t n = m - lo;
  return n >= 64u ? ~0ull : ((1ull << n) - 1ull);
}

__device__ __forceinline__ uint4 rec(uint64_t is0, uint64_t is1) {
  return make_uint4((uint32_t)is0, (uint32_t)(is0 >> 32), (uint32_t)is1, (uint32_t)(is1 >> 32));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// Ballot whose SGPR result may feed an inline-asm VALU (v_bcnt / v_writelane
// with an SGPR operand).  gfx950 needs 2 wait states between a VALU write of
// an SGPR/VCC and a VALU read of it; the compiler inserts them for its own
// instructions (s_nop 1 after v_cmp) but cannot see the read inside an asm
// statement.  The dependent s_nop below supplies them: every consumer of the
// returned mask is ordered after it.
__device__ __forceinline__ uint64_t ballot_s(bool p) {
  uint64_t b = __ballot(p);
  asm volatile("s_nop 1" : "+s"(b));
  return b;
}


// Coins of the tied receivers of one group (node.ts:111).  The key words are
// laundered through an empty asm so that Philox's ten round keys are not
// hoisted out of the round loop into permanently live SGPRs.
__device__ __forceinline__ uint64_t coin_ballot(uint32_t k0, uint32_t k1, uint32_t tlo, uint32_t thi,
                                             const uint32_t *__restrict__ live_ids, uint32_t group,
                                             uint32_t round, uint64_t tie) {
  const uint32_t lane = threadIdx.x & 63u;
  asm volatile("" : "+s"(k0), "+s"(k1));
  bool c1 = false;
  if ((tie >> lane) & 1ull) {
    const uint32_t node = live_ids[group * 64u + lane];
    const uint4 rr = philox4x32_10(k0, k1, make_uint4(tlo, thi, node, (round & 0x00FFFFFFu) | (kStreamCoin << 24)));
    c1 = !(rr.x > 0x80000000u);                 // Math.random() > 0.5 ? 0 : 1
  }
  return ballot(c1) & tie;
}

// Philox key words re-read from LDS at the point of use.  The volatile load
// cannot be hoisted, so the key schedule of a rare path (coins, the per-batch
// init pass) is rebuilt there instead of being kept -- i.e. spilled -- in SGPRs
// across the whole round loop.
__device__ __forceinline__ uint2 lds_keys(const uint32_t *keys) {
  const volatile __attribute__((address_space(3))) uint32_t *k =
      (const volatile __attribute__((address_space(3))) uint32_t *)keys;   // ds_read, not a flat load
  return make_uint2((uint32_t)__builtin_amdgcn_readfirstlane((int)k[0]),
                    (uint32_t)__builtin_amdgcn_readfirstlane((int)k[1]));
}

__device__ __forceinline__ uint64_t coin_ballot(const uint32_t *keys, uint32_t tlo, uint32_t thi,
                                             const uint32_t *__restrict__ live_ids, uint32_t group,
                                             uint32_t round, uint64_t tie) {
  const uint2 k = lds_keys(keys);
  tlo = (uint32_t)__builtin_amdgcn_readfirstlane((int)tlo);   // wave-uniform trial id; the asm keeps
  thi = (uint32_t)__builtin_amdgcn_readfirstlane((int)thi);   // Philox's first product on this path
  asm volatile("" : "+s"(tlo), "+s"(thi));
  return coin_ballot(k.x, k.y, tlo, thi, live_ids, group, round, tie);
}

// A call's result comes back in VGPRs; the ballot is wave-uniform, so move it
// to SGPRs for the mask arithmetic that follows.
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return (uint64_t)hi << 32 | lo;
}

// ------------------------------------------- W-specialised kernel (m <= 1024)
// For networks of at most 1024 live nodes (W <= 16 receiver groups) the whole
// round is unrolled at compile time: every receiver group's tally chain is a
// register, the plane records are read with immediate LDS offsets, a phase's
// ballots are staged into one VGPR with v_writelane and stored by one
// ds_write_b32, and the per-group `decided` masks live in SGPRs.  Initial
// values of TB = 64 / ceil(W/2) consecutive trials of the wave are drawn by
// one Philox pass (every lane busy) into an LDS ring.
template <int N, int I = 0>
struct Unroll {
  template <class Fn>
  __device__ __forceinline__ static void run(Fn &&f) {
    if constexpr (I < N) {
      f(std::integral_constant<int, I>{});
      Unroll<N, I + 1>::run(f);
    }
  }
};

// First step of receiver group C's chain: popcount(word) + C.  The distinct
// immediate per group keeps the groups' (identical, in lockstep) chains from
// being merged; comparisons are bias-invariant and thresholds add C.
template <int C>
__device__ __forceinline__ uint32_t tally_first(uint32_t word) {
  uint32_t r;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(word), "i"(C));
  return r;
}



// R-phase tally of one receiver group set: c1 only.  A receiver's R-phase
// trigger fires with exactly m messages in its inbox (node.ts:52, len >= N-F,
// m = N-F live senders in lockstep); each is 0, 1 or "?", so
// c0 = m - c1 - c? (node.ts:56-62) and c? is 0 in every round but the first
// of a fixed-init run with "?" initial values (a plan constant there).  The x
// planes therefore carry only the is1 word: 2 dwords per group, read as
// 16-byte pairs of groups.
template <int W>
__device__ __forceinline__ void tally_x1(const uint2 *__restrict__ plane, uint32_t (&a1)[W]) {
  const uint4 *q4 = reinterpret_cast<const uint4 *>(plane);
  {
    const uint4 q = q4[0];
    Unroll<W>::run([&](auto gi) {
      constexpr int g = decltype(gi)::value;
      a1[g] = tally_first<g>(q.x);
    });
#pragma unroll
    for (int g = 0; g < W; ++g) a1[g] = tally(q.y, a1[g]);
    if constexpr (W > 1) {
#pragma unroll
      for (int g = 0; g < W; ++g) {
        a1[g] = tally(q.z, a1[g]);
        a1[g] = tally(q.w, a1[g]);
      }
    }
  }
#pragma unroll
  for (int w = 1; w < W / 2; ++w) {
    const uint4 s = q4[w];
#pragma unroll
    for (int g = 0; g < W; ++g) {
      a1[g] = tally(s.x, a1[g]);
      a1[g] = tally(s.y, a1[g]);
      a1[g] = tally(s.z, a1[g]);
      a1[g] = tally(s.w, a1[g]);
    }
  }
  if constexpr (W > 1 && (W & 1)) {
    const uint2 s = plane[W - 1];
#pragma unroll
    for (int g = 0; g < W; ++g) {
      a1[g] = tally(s.x, a1[g]);
      a1[g] = tally(s.y, a1[g]);
    }
  }
}

// Proposal planes can stay in SGPRs for the few hundred cycles between the
// R-phase ballots that produce them and the P-phase tallies that read them:
// v_bcnt_u32_b32 takes its word from an SGPR at the same issue rate, so this
// saves the four staging moves per receiver group of the R-phase.
template <int C>
__device__ __forceinline__ uint32_t tally_first_s(uint32_t word) {
  uint32_t r;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "s"(word), "i"(C));
  return r;
}

__device__ __forceinline__ uint32_t tally_s(uint32_t word, uint32_t acc) {
  uint32_t r;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "s"(word), "v"(acc));
  return r;
}

// Wave-uniform 64-bit value re-read from LDS at the point of use (volatile:
// the read stays where it is written, see the W kernel's parameter block).
typedef const volatile __attribute__((address_space(3))) uint32_t lds_cv_u32;

__device__ __forceinline__ uint64_t lds_u64(const uint32_t *w) {
  lds_cv_u32 *k = (lds_cv_u32 *)w;   // ds_read, not a flat load
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)k[0]);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)k[1]);
  return (uint64_t)hi << 32 | lo;
}

__device__ __forceinline__ uint32_t sgpr32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// Per-lane select by a wave lane mask: lanes whose bit is set take `b`
// (one v_cndmask_b32 with an SGPR mask; a C select would shift the mask by
// the lane id in 64-bit VALU ops).
__device__ __forceinline__ uint32_t select_lanes(uint32_t a, uint32_t b, uint64_t mask) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(mask));
  return r;
}

// Opaque wave compares (v_cmp -> SGPR lane mask).  asm volatile so that the
// compiler neither merges the decision pass's compares with the adopt pass's
// recomputation of them (which would keep 2W masks live across the pass and
// spill SGPRs) nor speculates them out of their branches.  The trailing
// s_nop 1 supplies the 2 wait states gfx950 needs between a VALU SGPR write
// and a VALU read of it inside a later asm (v_bcnt with an SGPR operand).
__device__ __forceinline__ uint64_t vcmp_gt(uint32_t v, uint32_t s) {   // lanes with v > s
  uint64_t r;
  asm volatile("v_cmp_gt_u32_e64 %0, %1, %2\n\ts_nop 1" : "=s"(r) : "v"(v), "s"(s));
  return r;
}
__device__ __forceinline__ uint64_t vcmp_lt(uint32_t v, uint32_t s) {   // lanes with v < s
  uint64_t r;
  asm volatile("v_cmp_lt_u32_e64 %0, %1, %2\n\ts_nop 1" : "=s"(r) : "v"(v), "s"(s));
  return r;
}


template <int L>
__device__ __forceinline__ uint32_t writelane(uint32_t v, uint32_t val) {
  asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(val), "i"(L));
  return v;
}

// Stage one group's two ballot words (4 dwords) into lanes 4g..4g+3 of v.
template <int G>
__device__ __forceinline__ uint32_t stage4(uint32_t v, uint64_t is0, uint64_t is1) {
  v = writelane<4 * G + 0>(v, (uint32_t)is0);
  v = writelane<4 * G + 1>(v, (uint32_t)(is0 >> 32));
  v = writelane<4 * G + 2>(v, (uint32_t)is1);
  v = writelane<4 * G + 3>(v, (uint32_t)(is1 >> 32));
  return v;
}

// One round's R-phase proposals (node.ts:63-69, from each receiver's c1 and the
// binary vote count M) fused with the P-phase tallies (node.ts:92-98), for K
// independent trials at once (K > 1: small W, interleaved sender group by
// sender group so one trial's compares and tallies fill the other's
// dependency stalls).  Sender group w's proposal masks are added to every
// receiver group's counts as soon as they exist, so only one group's
// proposal planes (SGPR pairs) is live.
//
// ODD (M odd): c0 == c1 is impossible in the R-phase, so "c0 > c1" is the
// complement of "c1 > c0" (one compare) and no proposal is "?".  Every
// P-phase vote is then 0 or 1, so a receiver's c0 = m - c1 and only the c1
// tally is made (a0 is left unset; decide_k / the adopt pass derive it).
template <bool ODD, int W, int K>
__device__ __forceinline__ void p_phase_k(const uint32_t (&c1r)[K][W], uint32_t M, uint64_t tailm,
                                          uint32_t (&a0)[K][W], uint32_t (&a1)[K][W]) {
  const uint32_t hi_t = M >> 1, lo_t = (M + 1u) >> 1;
  Unroll<W>::run([&](auto wi) {
    constexpr int w = decltype(wi)::value;
    const uint64_t vm = (w == W - 1) ? tailm : ~0ull;
    Unroll<K>::run([&](auto ki) {
      constexpr int k = decltype(ki)::value;
      const uint64_t p1 = vcmp_gt(c1r[k][w], hi_t + (uint32_t)w) & vm;         // c1 > c0  (node.ts:65-66)
      const uint32_t l1 = (uint32_t)p1, h1 = (uint32_t)(p1 >> 32);
      if constexpr (!ODD) {
        const uint64_t p0 = vcmp_lt(c1r[k][w], lo_t + (uint32_t)w) & vm;       // c0 > c1  (node.ts:63-64), else "?"
        const uint32_t l0 = (uint32_t)p0, h0 = (uint32_t)(p0 >> 32);
        if constexpr (w == 0) {
          Unroll<W>::run([&](auto gi) {
            constexpr int g = decltype(gi)::value;
            a0[k][g] = tally_first_s<g>(l0);
          });
        } else {
#pragma unroll
          for (int g = 0; g < W; ++g) a0[k][g] = tally_s(l0, a0[k][g]);
        }
#pragma unroll
        for (int g = 0; g < W; ++g) a0[k][g] = tally_s(h0, a0[k][g]);
      }
      if constexpr (w == 0) {
        Unroll<W>::run([&](auto gi) {
          constexpr int g = decltype(gi)::value;
          a1[k][g] = tally_first_s<g>(l1);
        });
      } else {
#pragma unroll
        for (int g = 0; g < W; ++g) a1[k][g] = tally_s(l1, a1[k][g]);
      }
#pragma unroll
      for (int g = 0; g < W; ++g) a1[k][g] = tally_s(h1, a1[k][g]);
    });
  });
}

// Decisions (node.ts:99-105) of K trials: whether some live receiver stays
// undecided, and which values were decided.  ODD: c0 = m - c1, so
// "c0 > F" is "c1 < m - F" (no c0 tally exists).  Chain bias g throughout.
template <bool ODD, int W, int K>
__device__ __forceinline__ void decide_k(const uint32_t (&a0)[K][W], const uint32_t (&a1)[K][W], uint32_t m,
                                         uint32_t F, uint64_t tailm, uint64_t (&rest_any)[K], uint64_t (&any0)[K],
                                         uint64_t (&any1)[K]) {
  const uint32_t mF = m > F ? m - F : 0u;
#pragma unroll
  for (int k = 0; k < K; ++k) rest_any[k] = any0[k] = any1[k] = 0;
  Unroll<W>::run([&](auto gi) {
    constexpr int g = decltype(gi)::value;
    const uint64_t vm = (g == W - 1) ? tailm : ~0ull;
    Unroll<K>::run([&](auto ki) {
      constexpr int k = decltype(ki)::value;
      const uint64_t d0 = (ODD ? vcmp_lt(a1[k][g], mF + (uint32_t)g)           // node.ts:99
                               : vcmp_gt(a0[k][g], F + (uint32_t)g)) & vm;
      const uint64_t d1 = vcmp_gt(a1[k][g], F + (uint32_t)g) & vm & ~d0;      // node.ts:102
      rest_any[k] |= vm & ~(d0 | d1);
      any0[k] |= d0;
      any1[k] |= d1;
      // fold now: otherwise the ORs sink to the loop exit and all 2W masks stay live
      asm volatile("" : "+s"(rest_any[k]), "+s"(any0[k]), "+s"(any1[k]));
    });
  });
}

// STATE: the network API's single-trial launch that also reports per-node
// state and the halting round (GET /getState); the batch path is compiled
// without that code, which keeps its register allocation free of it.
constexpr int kPairMaxW = 8;               // W kernel: pair trials' round 1 up to this W

template <int W, bool STATE>
__global__ void __launch_bounds__(256) benor_lockstep_w_kernel(KParams p) {
  constexpr int NPH = (W + 1) / 2;          // Philox blocks per trial (2 plane words each)
  constexpr int TB = 64 / NPH;              // trials per init batch
  constexpr int WP = 2 * NPH;               // x1 words per plane row, padded to 16 bytes
  constexpr int K = W <= 2 ? 4 : (W <= kPairMaxW ? 2 : 1);   // trials whose round 1 runs interleaved
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // uniform: scalar trial loop
  // Only the round loop's own scalars are kept in registers.  What a rare
  // path needs (Philox key, trial id base, live ids) sits in a small LDS
  // parameter block and is re-read where it is used, so the register
  // allocator never holds -- and spills -- a kernarg tuple across the
  // trial loop.
  uint32_t m = p.m, F = p.F, k_max = p.k_max, hist_len = p.hist_len;
  // trial offsets within the launch are 32-bit (the host splits launches at 2^31)
  uint32_t trial_count = (uint32_t)p.trial_count;
  asm volatile("" : "+s"(m), "+s"(F), "+s"(k_max), "+s"(hist_len), "+s"(trial_count));

  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint2 *ring = reinterpret_cast<uint2 *>(smem + p.hist_bytes + wv * p.wave_bytes);   // [TB][WP] x1 words
  uint2 *X = ring + TB * WP;       // [WP] final x1 plane (GET /getState only)
  uint2 *D = X + WP;               // [WP] sticky decided bits, kept only while some receiver is undecided
  // parameter block: [0,1] Philox key (seed), [2,3] trial_begin, [4,5] live_ids
  uint32_t *keys = reinterpret_cast<uint32_t *>(smem + p.hist_bytes - kParamBytes);

  for (uint32_t i = threadIdx.x; i < hist_len; i += blockDim.x) lhist[i] = 0u;
  if (threadIdx.x == 0) {
    keys[0] = (uint32_t)p.seed;
    keys[1] = (uint32_t)(p.seed >> 32);
    keys[2] = (uint32_t)p.trial_begin;
    keys[3] = (uint32_t)(p.trial_begin >> 32);
    keys[4] = (uint32_t)(uintptr_t)p.live_ids;
    keys[5] = (uint32_t)((uintptr_t)p.live_ids >> 32);
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
  for (uint32_t base = blockIdx.x * kWavesPerBlock + wv; base < trial_count; base += waves_total * TB) {
    // ---- /start (node.ts:167-188): round-1 x planes of TB trials at once.
    if (random_init) {
      const uint32_t s = lane / NPH, b = lane - s * NPH;
      const uint32_t t = base + s * waves_total;
      if (s < (uint32_t)TB && t < trial_count) {
        const uint64_t trial = lds_u64(keys + 2) + t;
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
        const bool odd = M & 1u;
        if (odd) {
          p_phase_k<true, W, 1>(c1v, M, tailm, a0, a1);
          decide_k<true, W, 1>(a0, a1, m, F, tailm, rest_any, any0_, any1_);
        } else {
          p_phase_k<false, W, 1>(c1v, M, tailm, a0, a1);
          decide_k<false, W, 1>(a0, a1, m, F, tailm, rest_any, any0_, any1_);
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
          const uint32_t a0g = odd ? (m + 2u * (uint32_t)g) - a1[0][g] : a0[0][g];
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
              const uint64_t trial = lds_u64(keys + 2) + t;
              const uint32_t *ids = reinterpret_cast<const uint32_t *>((uintptr_t)lds_u64(keys + 4));
              x1 |= coin_ballot(keys, (uint32_t)trial, (uint32_t)(trial >> 32), ids, g, r, tie);
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
        if (s + K - 1 < TB && t + (uint32_t)(K - 1) * waves_total < trial_count) {
          // ---- round 1 of K trials interleaved; a trial that does not halt in
          // round 1 (some receiver undecided) is re-run alone from round 1.
          uint32_t c1[K][W], a0[K][W], a1[K][W];
          Unroll<K>::run([&](auto ki) {
            constexpr int k = decltype(ki)::value;
            tally_x1<W>(random_init ? ring + (s + k) * WP : ring, c1[k]);
          });
          uint64_t rest_any[K], any0[K], any1[K];
          if (m_first & 1u) {
            p_phase_k<true, W, K>(c1, m_first, tailm, a0, a1);
            decide_k<true, W, K>(a0, a1, m, F, tailm, rest_any, any0, any1);
          } else {
            p_phase_k<false, W, K>(c1, m_first, tailm, a0, a1);
            decide_k<false, W, K>(a0, a1, m, F, tailm, rest_any, any0, any1);
          }
          slow = 0u;
          nk = K;
          Unroll<K>::run([&](auto ki) {
            constexpr int k = decltype(ki)::value;
            if (!rest_any[k]) record(any0[k], any1[k], 1u, true);
            else slow |= 1u << k;
          });
        }
      }
      for (; slow; slow &= slow - 1u) {         // one call site: the whole-trial loop is inlined once
        const uint32_t k = (uint32_t)__builtin_ctz(slow);
        single(s + (int)k, t + k * waves_total);
      }
      s += (int)nk;
    }
  }

  if (hc) atomicAdd(&lhist[lane], hc);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < hist_len; i += blockDim.x) {
    const uint32_t c = lhist[i];
    if (c) atomicAdd(&p.hist[i], (unsigned long long)c);
  }
}


// --------------------------------------------- blocked kernel (1024 < m <= 4096)
// Receiver groups are processed in NB blocks of G (NB = ceil(W/16), G =
// ceil(W/NB), padding < NB groups); the record loop over the W plane words is
// a runtime loop.  Per-lane `decided` bits live in registers (one word per
// block).  Otherwise as the W-specialised kernel.
template <int G>
__device__ __forceinline__ void tally_groups(const uint4 *__restrict__ plane, uint32_t W, uint32_t (&a0)[G],
                                             uint32_t (&a1)[G]) {
  const uint4 q = plane[0];
  Unroll<G>::run([&](auto gi) {
    constexpr int g = decltype(gi)::value;
    a0[g] = tally_first<g>(q.x);
    a1[g] = tally_first<g>(q.z);
  });
#pragma unroll
  for (int g = 0; g < G; ++g) {
    a0[g] = tally(q.y, a0[g]);
    a1[g] = tally(q.w, a1[g]);
  }
  uint32_t w = 1;
  for (; w + 1 < W; w += 2) {
    const uint4 u = plane[w];
    const uint4 v = plane[w + 1];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      a0[g] = tally(u.x, a0[g]);
      a1[g] = tally(u.z, a1[g]);
      a0[g] = tally(u.y, a0[g]);
      a1[g] = tally(u.w, a1[g]);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      a0[g] = tally(v.x, a0[g]);
      a1[g] = tally(v.z, a1[g]);
      a0[g] = tally(v.y, a0[g]);
      a1[g] = tally(v.w, a1[g]);
    }
  }
  if (w < W) {
    const uint4 u = plane[w];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      a0[g] = tally(u.x, a0[g]);
      a1[g] = tally(u.z, a1[g]);
      a0[g] = tally(u.y, a0[g]);
      a1[g] = tally(u.w, a1[g]);
    }
  }
}

// R-phase x1-only tally over the W words of a plane (runtime W, pairs of
// groups per 16-byte read; WP = W rounded up to even, padding words zero).
template <int G>
__device__ __forceinline__ void tally_groups_x1(const uint2 *__restrict__ plane, uint32_t W, uint32_t (&a1)[G]) {
  const uint4 *q4 = reinterpret_cast<const uint4 *>(plane);
  const uint4 q = q4[0];
  Unroll<G>::run([&](auto gi) {
    constexpr int g = decltype(gi)::value;
    a1[g] = tally_first<g>(q.x);
  });
#pragma unroll
  for (int g = 0; g < G; ++g) {
    a1[g] = tally(q.y, a1[g]);
    a1[g] = tally(q.z, a1[g]);
    a1[g] = tally(q.w, a1[g]);
  }
  const uint32_t np = (W + 1u) >> 1;
  for (uint32_t w = 1; w < np; ++w) {
    const uint4 s = q4[w];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      a1[g] = tally(s.x, a1[g]);
      a1[g] = tally(s.y, a1[g]);
      a1[g] = tally(s.z, a1[g]);
      a1[g] = tally(s.w, a1[g]);
    }
  }
}

// One block's R-phase proposals (node.ts:63-69) from the receivers' c1
// counts, staged as {p0.lo, p0.hi, p1.lo, p1.hi} records for the P-phase
// tallies of every block.  ODD: an odd number of binary votes cannot tie,
// so p0 is the complement of p1 (one compare per group).
template <bool ODD, int G>
__device__ __forceinline__ uint32_t stage_proposals(const uint32_t (&a1)[G], uint32_t b, uint32_t m, uint32_t M) {
  const uint32_t hi_t = M >> 1, lo_t = (M + 1u) >> 1;
  uint32_t st = 0;
  Unroll<G>::run([&](auto gi) {
    constexpr int g = decltype(gi)::value;
    const uint64_t vm = group_mask(b * G + g, m);
    const uint64_t p1 = vcmp_gt(a1[g], hi_t + (uint32_t)g) & vm;          // c1 > c0  (node.ts:65-66)
    const uint64_t p0 = ODD ? (vm & ~p1)                                   // c0 > c1  (node.ts:63-64)
                            : (vcmp_lt(a1[g], lo_t + (uint32_t)g) & vm);   // else "?"
    st = stage4<g>(st, p0, p1);
  });
  return st;
}

template <int G, bool STATE>
__global__ void __launch_bounds__(256) benor_lockstep_blocked_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // scalar trial loop
  // Round-loop scalars in registers; the rest re-read where used (as the W kernel).
  uint32_t m = p.m, F = p.F, W = p.W, NB = p.nblocks, k_max = p.k_max, hist_len = p.hist_len;
  uint32_t trial_count = (uint32_t)p.trial_count;     // launches are split at 2^31 trials
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
    keys[4] = (uint32_t)(uintptr_t)p.live_ids;
    keys[5] = (uint32_t)((uintptr_t)p.live_ids >> 32);
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
        const uint64_t trial = lds_u64(keys + 2) + t;
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
        auto round = [&](auto odd_c) {
          constexpr bool ODD = decltype(odd_c)::value;
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
              const uint32_t st = stage_proposals<false, G>(a1, b, m, M);
              if (lane < 4u * G) reinterpret_cast<uint32_t *>(P + b * G)[lane] = st;
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
            uint32_t st = 0, dbb = D[b * 64u + lane];
            Unroll<G>::run([&](auto gi) {
              constexpr int g = decltype(gi)::value;
              const uint64_t vm = group_mask(b * G + g, m);
              const uint32_t Fg = F + (uint32_t)g;
              const uint64_t d0 = (ODD ? vcmp_lt(a1[g], mF + (uint32_t)g)   // c0 = m - c1 > F
                                       : vcmp_gt(a0[g], Fg)) & vm;          // node.ts:99
              const uint64_t d1 = vcmp_gt(a1[g], Fg) & vm & ~d0;           // node.ts:102
              const uint64_t rest = vm & ~(d0 | d1);
              uint64_t x1 = d1;
              if (rest) {
                const uint32_t a0g = ODD ? (m + 2u * (uint32_t)g) - a1[g] : a0[g];   // bias g
                const uint64_t ad1 = ballot_s(a1[g] > a0g) & rest;         // node.ts:108-109
                const uint64_t tie = ballot_s(a1[g] == a0g) & rest;        // node.ts:110-111
                x1 |= ad1;
                if (tie) {                                                // node.ts:111
                  const uint64_t trial = lds_u64(keys + 2) + t;
                  const uint32_t *ids = reinterpret_cast<const uint32_t *>((uintptr_t)lds_u64(keys + 4));
                  x1 |= coin_ballot(keys, (uint32_t)trial, (uint32_t)(trial >> 32), ids, b * G + g, r, tie);
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
        if (M & 1u) round(std::true_type{});
        else round(std::false_type{});
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
  for (uint32_t i = threadIdx.x; i < hist_len; i += blockDim.x) {
    const uint32_t c = lhist[i];
    if (c) atomicAdd(&p.hist[i], (unsigned long long)c);
  }
}


// ------------------------------------------------ packed kernel (m <= 32)
// Small networks (BASELINE configs C1 N=5, C2 N=10, and the C5 sweep's small
// cells) would leave most of a wave idle with one trial per wave.  Here every
// 32-lane half of a wave holds P = floor(32/m) independent trials
// ("segments") of m lanes each, so one wave runs 2P trials concurrently:
//
//   * lane (h*32 + i*m + c) is live node c (compact order) of segment h*P + i;
//   * a phase's messages for all segments are ONE pair of wave ballots
//     {is0, is1}; each receiver tallies its own segment's bits:
//     popcount((ballot >> 32h) & segment_mask) per count;
//   * segments advance independently: when a segment's trial halts (every
//     live node decided, or k_max rounds), its leader lane records the
//     outcome and the segment pulls the wave's next trial from a per-wave
//     queue.  Random initial values for the queue come from an LDS ring of
//     128 words filled 64 trials per Philox pass (one trial per lane);
//   * coins (node.ts:111) are per lane, only on rounds where some receiver ties.
// Same outcome definition as the other lockstep kernels: the histogram is
// bit-identical to theirs (the trial -> wave assignment only changes order).
__device__ __forceinline__ uint32_t seg_tally(uint64_t plane, uint32_t half_shift, uint32_t segmask) {
  // one receiver's count over its segment's senders (node.ts:56-62, :92-98)
  return (uint32_t)__builtin_popcount((uint32_t)(plane >> half_shift) & segmask);
}

__global__ void __launch_bounds__(256) benor_packed_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t m = p.m, F = p.F;
  const uint32_t P = 32u / m;                       // segments per half
  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint32_t *ring = reinterpret_cast<uint32_t *>(smem + p.hist_bytes + wv * p.wave_bytes);   // [128]

  for (uint32_t i = threadIdx.x; i < p.hist_len; i += blockDim.x) lhist[i] = 0u;
  __syncthreads();

  const uint32_t hl = lane & 31u;
  const uint32_t si = hl / m;                       // segment index within the half
  const uint32_t c = hl - si * m;                   // compact live index of this lane's node
  const bool valid = si < P;
  const uint32_t half_shift = lane & 32u;
  const uint32_t mbits = m == 32u ? ~0u : ((1u << m) - 1u);
  const uint32_t segmask = valid ? (mbits << (si * m)) : 0u;
  const uint32_t node = valid ? p.live_ids[c] : 0u;
  const bool random_init = p.init_mode == BO_INIT_RANDOM;
  // fixed init (BO_INIT_FIXED): word 0 of the plane holds every live node (m <= 32)
  const uint4 fixed = random_init ? make_uint4(0, 0, 0, 0) : p.init_plane[0];
  const uint32_t fixed_x = ((fixed.z >> c) & 1u) ? 1u : (((fixed.x >> c) & 1u) ? 0u : 2u);

  const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
  const uint64_t gw = (uint64_t)blockIdx.x * kWavesPerBlock + wv;
  const uint64_t waves_total = (uint64_t)gridDim.x * kWavesPerBlock;

  uint64_t next_j = 0, filled = 0;                  // wave queue: j-th trial of the wave = gw + j * waves_total
  bool need = valid, act = false, dec = false;
  uint32_t x = 2u, r = 0u;
  uint64_t trial = 0;

  for (;;) {
    // ---- pull: segments that need a trial take the next queue entries (node.ts:167-188 /start)
    const uint64_t Lb = ballot(need && c == 0u);
    if (Lb) {
      const uint32_t nf = (uint32_t)__builtin_popcountll(Lb);
      if (random_init && next_j + nf > filled) {   // refill 64 ring slots, one trial per lane
        const uint64_t j = filled + lane;
        const uint64_t t = gw + j * waves_total;
        if (t < p.trial_count) {
          const uint64_t tr = p.trial_begin + t;
          uint32_t kk0 = k0, kk1 = k1;
          asm volatile("" : "+s"(kk0), "+s"(kk1));
          ring[j & 127u] = philox4x32_10(kk0, kk1, make_uint4((uint32_t)tr, (uint32_t)(tr >> 32), 0u, kStreamInit << 24)).x;
        }
        filled += 64u;
      }
      if (need) {
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(Lb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)Lb, 0u));
        const uint64_t j = next_j + below - (c ? 1u : 0u);
        const uint64_t t = gw + j * waves_total;
        need = false;
        act = t < p.trial_count;
        if (act) {
          trial = p.trial_begin + t;
          x = random_init ? ((ring[j & 127u] >> c) & 1u) : fixed_x;
          dec = false;
          r = 0u;
        }
      }
      next_j += nf;
    }
    if (!__any(act)) break;

    // ---- R-phase ("proposal phase", node.ts:46-82): c1 per receiver, c0 = M - c1
    //      (M = m binary-valued senders; minus the "?" ones in round 1 of a fixed init)
    const uint64_t is1 = ballot(act && x == 1u);
    const uint32_t c1 = seg_tally(is1, half_shift, segmask);
    const uint32_t c0 = (r == 0u ? m - p.init_q : m) - c1;
    // ---- P-phase ("voting phase", node.ts:83-158)
    const uint64_t p0 = ballot(act && c0 > c1), p1 = ballot(act && c1 > c0);   // node.ts:63-69 (else "?")
    const uint32_t v0 = seg_tally(p0, half_shift, segmask), v1 = seg_tally(p1, half_shift, segmask);
    ++r;
    const bool d0 = v0 > F, d1 = !d0 && v1 > F;                                    // node.ts:99, :102
    const bool tie = act && !d0 && !d1 && v0 == v1;                                // node.ts:110-111
    uint32_t nx = d0 ? 0u : (d1 ? 1u : (v1 > v0 ? 1u : 0u));                        // node.ts:106-109
    if (__any(tie)) {
      uint32_t kk0 = k0, kk1 = k1;
      asm volatile("" : "+s"(kk0), "+s"(kk1));
      if (tie) {
        const uint4 rr = philox4x32_10(kk0, kk1, make_uint4((uint32_t)trial, (uint32_t)(trial >> 32), node,
                                                            (r & 0x00FFFFFFu) | (kStreamCoin << 24)));
        nx = (rr.x > 0x80000000u) ? 0u : 1u;                                       // Math.random() > 0.5 ? 0 : 1
      }
    }
    if (act) {
      x = nx;
      dec = dec || d0 || d1;                                                        // sticky (node.ts:100-105)
    }
    // ---- halt: every live node of the segment decided (auto-stop, node.ts:116-145) or k_max
    const uint64_t db = ballot(act && dec);
    const bool seg_done = seg_tally(db, half_shift, segmask) == m;
    const bool fin = act && (seg_done || r >= p.k_max);
    if (__any(fin)) {
      const uint64_t n0 = ballot(act && x == 0u), n1 = ballot(act && x == 1u);
      if (fin) {
        const bool any0 = seg_tally(n0, half_shift, segmask) != 0u, any1 = seg_tally(n1, half_shift, segmask) != 0u;
        const uint32_t v = (any0 && any1) ? 2u : (any1 ? 1u : 0u);
        if (c == 0u) {
          atomicAdd(&lhist[seg_done ? (r * 3u + v) : v], 1u);
          if (seg_done && v == 2u) atomicAdd(&lhist[p.hist_len - 1u], 1u);
          if (p.rounds_out) *p.rounds_out = seg_done ? r : 0u;
        }
        if (p.node_out) {                                                           // GET /getState (node.ts:197-199)
          bo_node_state ns;
          ns.killed = 0;
          ns.x = (int8_t)x;
          ns.decided = (int8_t)(dec ? 1 : 0);
          ns.pad = 0;
          ns.k = (int32_t)r + 1;                                                    // node.ts:147
          p.node_out[node] = ns;
        }
        act = false;
        need = true;
      }
    }
  }

  __syncthreads();
  for (uint32_t i = threadIdx.x; i < p.hist_len; i += blockDim.x) {
    const uint32_t cnt = lhist[i];
    if (cnt) atomicAdd(&p.hist[i], (unsigned long long)cnt);
  }
}


// ----------------------------------------- random-delivery kernel (f <= F)
// Generalised delivery: with f <= F crashed nodes every live
// receiver tallies, per phase, a uniformly random subset of exactly q = N-F of
// the m = N-f live senders ("first N-F arrivals"), drawn by Floyd's algorithm
// from Philox stream 2 (definition: oracle/benor_oracle.c
// oracle_delivery_mask).  The subset is built per lane in an LDS bitset laid
// out [word][lane] (any per-lane word index is bank-conflict free), then the
// receiver's inbox is (sender plane AND delivery mask).  One receiver group
// (64 receivers) at a time; this mode is bound by the subset's random draws.
struct DStream {
  uint32_t k0, k1, c0, c1, c2, c3;
  uint4 buf;
  uint32_t widx;
  __device__ __forceinline__ uint32_t next() {
    if ((widx & 3u) == 0u) buf = philox4x32_10(k0, k1, make_uint4(c0, c1, c2 | ((widx >> 2) << 12), c3));
    const uint32_t j = widx & 3u;
    ++widx;
    return j == 0 ? buf.x : j == 1 ? buf.y : j == 2 ? buf.z : buf.w;
  }
  // uniform in [0, range): Lemire's multiply-shift with exact rejection
  __device__ __forceinline__ uint32_t uniform(uint32_t range) {
    uint64_t mm = (uint64_t)next() * range;
    uint32_t l = (uint32_t)mm;
    if (l < range) {
      const uint32_t t = (0u - range) % range;
      while (l < t) {
        mm = (uint64_t)next() * range;
        l = (uint32_t)mm;
      }
    }
    return (uint32_t)(mm >> 32);
  }
};

// One Floyd step: sender t, else (t already in the subset) sender jj, joins
// the lane's bitset ([word][lane] in LDS).  ds_or: LDS ops of a wave retire
// in order, so the next step's read sees this one.
__device__ __forceinline__ void floyd_insert(uint32_t *__restrict__ B, uint32_t lane, uint32_t t, uint32_t jj) {
  const uint32_t cur = B[(t >> 5) * 64u + lane];
  const uint32_t idx = ((cur >> (t & 31u)) & 1u) ? jj : t;
  atomicOr(&B[(idx >> 5) * 64u + lane], 1u << (idx & 31u));
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
  const uint32_t c2 = node & 0xFFFu, c3 = (r & 0xFFFFFu) | ((phase & 1u) << 20) | (kStreamDelivery << 24);
  uint32_t jj = m - k, widx = 0;
  for (;;) {
    const bool go = active && jj < m;
    if (!__any(go)) break;
    bool fast = go && (widx & 3u) == 0u;
    if (fast) {
      const uint4 b = philox4x32_10(k0, k1, make_uint4(tlo, thi, c2 | ((widx >> 2) << 12), c3));
      const uint32_t n = m - jj < 4u ? m - jj : 4u;            // draws left in this subset
      const uint64_t q0 = (uint64_t)b.x * (jj + 1u), q1 = (uint64_t)b.y * (jj + 2u);
      const uint64_t q2 = (uint64_t)b.z * (jj + 3u), q3 = (uint64_t)b.w * (jj + 4u);
      const bool rej = (uint32_t)q0 < jj + 1u || (n > 1u && (uint32_t)q1 < jj + 2u) ||
                       (n > 2u && (uint32_t)q2 < jj + 3u) || (n > 3u && (uint32_t)q3 < jj + 4u);
      if (!rej) {
        floyd_insert(B, lane, (uint32_t)(q0 >> 32), jj);
        if (n > 1u) floyd_insert(B, lane, (uint32_t)(q1 >> 32), jj + 1u);
        if (n > 2u) floyd_insert(B, lane, (uint32_t)(q2 >> 32), jj + 2u);
        if (n > 3u) floyd_insert(B, lane, (uint32_t)(q3 >> 32), jj + 3u);
        jj += n;
        widx += n;
      } else {
        fast = false;
      }
    }
    if (go && !fast) {
      DStream ds;
      ds.k0 = k0; ds.k1 = k1; ds.c0 = tlo; ds.c1 = thi; ds.c2 = c2; ds.c3 = c3;
      ds.widx = widx & ~3u;                                      // refill the current block, then skip to widx
      for (uint32_t i = ds.widx; i < widx; ++i) (void)ds.next();
      const uint32_t t = ds.uniform(jj + 1u);
      floyd_insert(B, lane, t, jj);
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
        const uint4 r = philox4x32_10(k0, k1, make_uint4(tlo, thi, lane, kStreamInit << 24));
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
          if (tie) x1 |= coin_ballot(k0, k1, tlo, thi, p.live_ids, j, r, tie);
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
  for (uint32_t i = threadIdx.x; i < p.hist_len; i += blockDim.x) {
    const uint32_t c = lhist[i];
    if (c) atomicAdd(&p.hist[i], (unsigned long long)c);
  }
}


// ------------------------------------------------ event-level kernel (N <= 64)
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

struct EvLane {
  uint32_t *pool;      // [cap]
  uint32_t *ibox;      // [N][4][2] packed {c0, c1, len} bytes
  int8_t *xs;          // [N]
  int16_t *ks;         // [N]
  uint64_t *comp;      // [4] completion masks, round k at k & 3
  uint32_t *crash;     // [64] sorted (event << 6 | node)
};

__global__ void __launch_bounds__(256) benor_event_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  for (uint32_t i = threadIdx.x; i < p.hist_len; i += blockDim.x) lhist[i] = 0u;
  __syncthreads();

  const uint32_t N = p.N, F = p.F, quorum = p.N - p.F, m = p.m;
  const uint64_t all = N == 64 ? ~0ull : ((1ull << N) - 1ull);
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
  const uint32_t cap = p.ev_cap;
  uint32_t *base = p.scratch + gid * p.ev_stride;
  EvLane L;
  L.pool = base;
  L.ibox = L.pool + cap;
  L.comp = reinterpret_cast<uint64_t *>(L.ibox + N * 8u);
  L.crash = reinterpret_cast<uint32_t *>(L.comp + 4);
  L.xs = reinterpret_cast<int8_t *>(L.crash + 64);
  L.ks = reinterpret_cast<int16_t *>(L.xs + 64);
  const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);

  for (uint64_t t = gid; t < p.trial_count; t += lanes) {
    const uint64_t trial = p.trial_begin + t;
    const uint32_t tlo = (uint32_t)trial, thi = (uint32_t)(trial >> 32);
    uint64_t killed = p.faulty_mask, decided = 0;
    // ---- node.ts:21-26 and initial values (compact live order)
    uint4 ir = make_uint4(0, 0, 0, 0);
    if (p.init_mode == BO_INIT_RANDOM) ir = philox4x32_10(k0, k1, make_uint4(tlo, thi, 0u, kStreamInit << 24));
    for (uint32_t c = 0; c < m; ++c) {
      const uint32_t i = p.live_ids[c];
      int8_t v;
      if (p.init_mode == BO_INIT_RANDOM) v = (int8_t)((((c >> 5) ? ir.y : ir.x) >> (c & 31u)) & 1u);
      else v = p.init_x[i];
      L.xs[i] = v;
      L.ks[i] = 0;
    }
    for (uint32_t i = 0; i < N; ++i)
      if ((killed >> i) & 1ull) { L.xs[i] = -1; L.ks[i] = -1; }
    for (uint32_t j = 0; j < N * 8u; ++j) L.ibox[j] = 0u;
    for (int j = 0; j < 4; ++j) L.comp[j] = 0ull;
    // ---- mid-run /stop schedule, sorted by event index
    uint32_t ncrash = 0;
    if (p.crash_at) {
      for (uint32_t i = 0; i < N; ++i)
        if (p.crash_at[i] != 0xFFFFFFFFu && p.crash_at[i] < (1u << 26)) L.crash[ncrash++] = (p.crash_at[i] << 6) | i;
    } else if (p.crash_count > 0 && m > 0 && p.crash_window > 0) {
      DStream ds;
      ds.k0 = k0; ds.k1 = k1; ds.c0 = tlo; ds.c1 = thi; ds.c2 = 0u; ds.c3 = kStreamCrash << 24; ds.widx = 0;
      const uint32_t kk = p.crash_count < m ? p.crash_count : m;
      uint64_t T = 0;
      uint32_t picks[64];
      uint32_t n = 0;
      for (uint32_t j = m - kk; j < m; ++j, ++n) {
        const uint32_t tt = ds.uniform(j + 1u);
        const uint32_t idx = ((T >> tt) & 1ull) ? j : tt;
        T |= 1ull << idx;
        picks[n] = idx;
      }
      for (uint32_t q2 = 0; q2 < kk; ++q2) {
        const uint32_t when = ds.uniform(p.crash_window);
        if (when < (1u << 26)) L.crash[ncrash++] = (when << 6) | p.live_ids[picks[q2]];
      }
    }
    for (uint32_t a = 1; a < ncrash; ++a) {            // insertion sort (<= 64 entries)
      const uint32_t v = L.crash[a];
      uint32_t b = a;
      while (b > 0 && L.crash[b - 1] > v) { L.crash[b] = L.crash[b - 1]; --b; }
      L.crash[b] = v;
    }
    uint32_t next = 0;
    // ---- delivery order
    uint64_t rng;
    {
      const uint4 o = philox4x32_10(k0, k1, make_uint4(tlo, thi, 0u, kStreamOrder << 24));
      rng = (((uint64_t)o.x << 32) | o.y) ^ 0xD1B54A32D192ED03ull;
    }
    // ---- /start (node.ts:167-188)
    uint32_t len = 0;
    for (uint32_t i = 0; i < N; ++i) {
      if ((killed >> i) & 1ull) continue;
      L.ks[i] = 1;
      const uint32_t body = ((uint32_t)(L.xs[i] & 3) << 7) | (1u << 9);
      for (uint32_t to = 0; to < N; ++to) L.pool[len++] = to | body;
    }
    uint32_t cur = 1, R = 0, halted = 0;
    bool overflow = false;
    for (uint32_t e = 0;; ++e) {
      // scheduled GET /stop (node.ts:191-194)
      bool crashed = false;
      while (next < ncrash && (L.crash[next] >> 6) == e) {
        const uint32_t i = L.crash[next] & 63u;
        killed |= 1ull << i;
        crashed = true;
        ++next;
      }
      if (crashed) {
        if (killed == all) { halted = 3; break; }
        while ((L.comp[cur & 3u] | killed) == all) {
          if ((decided | killed) == all) { halted = 1; R = cur; break; }
          if (cur >= p.k_max) { halted = 2; R = cur; break; }
          L.comp[cur & 3u] = 0ull;
          ++cur;
        }
        if (halted) break;
      }
      if (len == 0) { halted = 3; break; }
      const uint32_t pick = (uint32_t)(((uint64_t)(uint32_t)(splitmix64(rng) >> 32) * (uint64_t)len) >> 32);
      const uint32_t msg = L.pool[pick];
      L.pool[pick] = L.pool[--len];
      const uint32_t to = msg & 63u, ph = (msg >> 6) & 1u, k = msg >> 9;
      const uint32_t x = (msg >> 7) & 3u;
      if ((killed >> to) & 1ull) continue;             // node.ts:45
      uint32_t *bx = &L.ibox[(to * 4u + (k & 3u)) * 2u + ph];
      uint32_t b = *bx;
      b += 1u << 16;                                   // len
      if (x == 0u) b += 1u;                            // c0
      else if (x == 1u) b += 1u << 8;                  // c1
      *bx = b;
      if ((b >> 16) != quorum) continue;               // node.ts:52, :88 (fires once: exactly F faulty)
      const uint32_t c0 = b & 0xFFu, c1 = (b >> 8) & 0xFFu;
      uint32_t body;
      if (ph == 0u) {                                  // node.ts:53-80
        const uint32_t v = c0 > c1 ? 0u : (c1 > c0 ? 1u : 2u);
        body = (1u << 6) | (v << 7) | (k << 9);
      } else {                                         // node.ts:89-157
        int8_t nx;
        if (c0 > F) { nx = 0; decided |= 1ull << to; }
        else if (c1 > F) { nx = 1; decided |= 1ull << to; }
        else if (c0 + c1 > 0 && c0 > c1) nx = 0;
        else if (c0 + c1 > 0 && c0 < c1) nx = 1;
        else {
          const uint4 rr = philox4x32_10(k0, k1, make_uint4(tlo, thi, to, (k & 0x00FFFFFFu) | (kStreamCoin << 24)));
          nx = (rr.x > 0x80000000u) ? 0 : 1;           // node.ts:111
        }
        L.xs[to] = nx;
        L.ks[to] = (int16_t)(k + 1u);
        L.ibox[(to * 4u + ((k + 2u) & 3u)) * 2u + 0u] = 0u;   // recycle round k-2's slots for k+2
        L.ibox[(to * 4u + ((k + 2u) & 3u)) * 2u + 1u] = 0u;
        L.comp[k & 3u] |= 1ull << to;
        while ((L.comp[cur & 3u] | killed) == all) {
          if ((decided | killed) == all) { halted = 1; R = cur; break; }
          if (cur >= p.k_max) { halted = 2; R = cur; break; }
          L.comp[cur & 3u] = 0ull;
          ++cur;
        }
        if (halted) break;
        body = ((uint32_t)(nx & 3) << 7) | ((k + 1u) << 9);
      }
      if (len + N > cap) { overflow = true; halted = 3; break; }
      for (uint32_t dst = 0; dst < N; ++dst) L.pool[len++] = dst | body;
    }
    // ---- outcome over the nodes still running
    bool any0 = false, any1 = false, anyq = false;
    uint32_t nlive = 0;
    for (uint32_t i = 0; i < N; ++i) {
      if ((killed >> i) & 1ull) continue;
      ++nlive;
      const int8_t v = L.xs[i];
      if (v == 0) any0 = true; else if (v == 1) any1 = true; else anyq = true;
    }
    const uint32_t v = (nlive == 0 || anyq || (any0 && any1)) ? 2u : (any1 ? 1u : 0u);
    atomicAdd(&lhist[halted == 1 ? (R * 3u + v) : v], 1u);
    if (halted == 1 && v == 2u) atomicAdd(&lhist[p.hist_len - 1u], 1u);
    if (overflow && p.rounds_out) atomicOr(p.rounds_out, 0x80000000u);
    if (p.node_out) {
      for (uint32_t i = 0; i < N; ++i) {
        const bool f = (p.faulty_mask >> i) & 1ull;
        bo_node_state ns;
        ns.killed = (int8_t)((killed >> i) & 1ull);
        ns.x = L.xs[i];
        ns.decided = f ? (int8_t)-1 : (int8_t)((decided >> i) & 1ull);
        ns.pad = 0;
        ns.k = L.ks[i];
        p.node_out[i] = ns;
      }
      if (p.rounds_out) atomicOr(p.rounds_out, halted == 1 ? R : 0u);
    }
  }

  __syncthreads();
  for (uint32_t i = threadIdx.x; i < p.hist_len; i += blockDim.x) {
    const uint32_t c = lhist[i];
    if (c) atomicAdd(&p.hist[i], (unsigned long long)c);
  }
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
  if (p.mode == BO_MODE_EVENT) {
    p.G = 1;
    p.nblocks = 1;
    p.variant = 4;
    p.wave_bytes = 0;
    p.lds_bytes = p.hist_bytes;
    // per-lane scratch (u32 words): pool, inbox window, comp[4] (u64), crash[64], xs[64] (i8), ks[64] (i16)
    p.ev_cap = 4u * p.N * p.N + 64u;
    p.ev_stride = p.ev_cap + p.N * 8u + 8u + 64u + 16u + 32u;
    p.ev_stride = (p.ev_stride + 31u) & ~31u;
    return;
  }
  if (p.mode == BO_MODE_RANDOM_DELIVERY) {
    p.G = 1;
    p.nblocks = W;
    p.variant = 2;
    p.wave_bytes = 2u * W * 16u + 2u * W * 64u * 4u;   // X, P records + per-lane bitset
    p.lds_bytes = p.hist_bytes + kWavesPerBlock * p.wave_bytes;
    return;
  }
  if (p.m <= kMaxPackedM) {                         // packed: floor(32/m) trials per half-wave
    p.G = 1;
    p.nblocks = 1;
    p.variant = 5;
    p.wave_bytes = 128u * 4u;                       // init-word ring
    p.lds_bytes = p.hist_bytes + kWavesPerBlock * p.wave_bytes;
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
    const uint32_t nb = (W + 15u) / 16u;           // blocks of at most 16 groups
    const uint32_t G = (W + nb - 1u) / nb;         // balanced: padding < nb groups
    const uint32_t XW = ((G * nb > WP ? G * nb : WP) + 1u) & ~1u;
    p.G = G;
    p.nblocks = nb;
    p.variant = 0;
    p.wave_bytes = (tb * WP + XW) * 8u + G * nb * 16u + nb * 256u;   // ring, x1 plane, {p0,p1} plane, decided bits
  }
  p.lds_bytes = p.hist_bytes + kWavesPerBlock * p.wave_bytes;
}

template <int W>
static hipError_t launch_w(const KParams &p, int grid, hipStream_t s) {
  if (p.node_out || p.rounds_out)
    hipLaunchKernelGGL((benor_lockstep_w_kernel<W, true>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  else
    hipLaunchKernelGGL((benor_lockstep_w_kernel<W, false>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  return hipGetLastError();
}

template <int G>
static hipError_t launch_b(const KParams &p, int grid, hipStream_t s) {
  if (p.node_out || p.rounds_out)
    hipLaunchKernelGGL((benor_lockstep_blocked_kernel<G, true>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  else
    hipLaunchKernelGGL((benor_lockstep_blocked_kernel<G, false>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  return hipGetLastError();
}

template <int... Is>
static hipError_t dispatch_w(const KParams &p, int grid, hipStream_t s, std::integer_sequence<int, Is...>) {
  hipError_t e = hipErrorInvalidValue;
  (void)((p.W == (uint32_t)(Is + 1) ? (e = launch_w<Is + 1>(p, grid, s), true) : false) || ...);
  return e;
}

// W in 17..64: G = ceil(W / ceil(W/16)) in 9..16
template <int... Is>
static hipError_t dispatch_b(const KParams &p, int grid, hipStream_t s, std::integer_sequence<int, Is...>) {
  hipError_t e = hipErrorInvalidValue;
  (void)((p.G == (uint32_t)(Is + 9) ? (e = launch_b<Is + 9>(p, grid, s), true) : false) || ...);
  return e;
}

hipError_t launch_lockstep(const KParams &p, int grid, hipStream_t s) {
  if (p.variant == 4) {
    hipLaunchKernelGGL(benor_event_kernel, dim3(grid), dim3(256), p.lds_bytes, s, p);
    return hipGetLastError();
  }
  if (p.variant == 5) {
    hipLaunchKernelGGL(benor_packed_kernel, dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
    return hipGetLastError();
  }
  if (p.variant == 2) {
    if (p.lds_bytes > 64u * 1024u) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&benor_random_kernel),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds_bytes);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(benor_random_kernel, dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
    return hipGetLastError();
  }
  if (p.variant == 1) return dispatch_w(p, grid, s, std::make_integer_sequence<int, kMaxWSpecialised>{});
  return dispatch_b(p, grid, s, std::make_integer_sequence<int, 8>{});
}

int lockstep_grid(const KParams &p, int device) {
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (p.variant == 4) {   // event mode: one lane per trial, grid = the scratch's lane count
    const uint64_t blocks_needed = (p.trial_count + 255u) / 256u;
    uint64_t grid = p.ev_lanes / 256u;
    if (blocks_needed < grid) grid = blocks_needed;
    return (int)(grid < 1 ? 1 : grid);
  }
  // 8 workgroups (32 waves) per CU when registers and LDS allow it.
  const uint64_t per_wave = p.variant == 5 ? 2u * (32u / p.m) : 1u;   // trials a wave runs at once
  const uint64_t waves_needed = (p.trial_count + per_wave - 1u) / per_wave;
  const uint64_t blocks_needed = (waves_needed + kWavesPerBlock - 1) / kWavesPerBlock;
  uint64_t per_cu = 8;
  if (p.lds_bytes > 0) {
    const uint64_t lds_fit = (160u * 1024u) / p.lds_bytes;
    if (lds_fit < per_cu) per_cu = lds_fit ? lds_fit : 1;
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
