// benor_device.h -- device-side building blocks shared by the gfx950 round-loop
// kernels (benor_kernels.hip, benor_w_*.hip, benor_blocked.hip): Philox4x32-10,
// opaque per-receiver tallies, wave compares and ballots, lane staging, and
// the W kernel's fused R/P phase.  See benor_kernels.hip for the design notes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "benor_internal.h"

namespace benor {

// ------------------------------------------------------------------ Philox
// hi ^ c ^ key in one gfx950 v_bitop3_b32 (LUT 0x96 = three-way xor; the key is
// wave-uniform: an SGPR operand).
// Left to itself the compiler emits two v_xor_b32 per output word.
__device__ __forceinline__ uint32_t xor3_key(uint32_t hi, uint32_t c, uint32_t key) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(hi), "v"(c), "s"(key));
  return r;
}

// 32x32 -> 64-bit product in one v_mad_u64_u32 (m wave-uniform).  It issues
// at ~4.9 cycles per wave64 instruction against ~8.4 for the v_mul_lo_u32 +
// v_mul_hi_u32 pair the compiler picks (tools/valu_probe.hip).  The unused
// carry-out goes to VCC (a fresh SGPR pair per product raised SGPR pressure
// to spilling in the event kernel).
__device__ __forceinline__ uint64_t mul_wide(uint32_t a, uint32_t m) {
  uint64_t r;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(a), "s"(m) : "vcc");
  return r;
}

// Philox4x32-10 (Salmon et al., SC'11; Random123).  Callers pass a
// wave-uniform key (the seed); the counter may vary per lane.  WIDE: the
// products by v_mad_u64_u32 (throughput-bound callers); otherwise by
// v_mul_lo/v_mul_hi pairs, whose shorter dependency chain suits the
// latency-bound event kernel (13 % faster there).
template <bool WIDE = true>
__device__ __forceinline__ uint4 philox4x32_10(uint32_t k0, uint32_t k1, uint4 c) {
  k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k0);    // no-op on an SGPR key
  k1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k1);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t lo0, hi0, lo1, hi1;
    if constexpr (WIDE) {
      const uint64_t p0 = mul_wide(c.x, 0xD2511F53u);
      const uint64_t p1 = mul_wide(c.z, 0xCD9E8D57u);
      lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
      lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    } else {
      lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
      lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    }
    c = make_uint4(xor3_key(hi1, c.y, k0), lo1, xor3_key(hi0, c.w, k1), lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Philox4x32-10 of K counters at once, round by round, so that the K
// independent dependency chains interleave in the instruction stream (one
// wave computing several blocks is otherwise latency-bound on the products).
template <int K>
__device__ __forceinline__ void philox4x32_10_multi(uint32_t k0, uint32_t k1, uint4 (&c)[K]) {
  k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k0);
  k1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k1);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const uint64_t p0 = mul_wide(c[i].x, 0xD2511F53u);
      const uint64_t p1 = mul_wide(c[i].z, 0xCD9E8D57u);
      c[i] = make_uint4(xor3_key((uint32_t)(p1 >> 32), c[i].y, k0), (uint32_t)p1,
                        xor3_key((uint32_t)(p0 >> 32), c[i].w, k1), (uint32_t)p0);
    }
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// Sequential word stream of Philox blocks (oracle orc_dstream): word i is
// element i & 3 of block i >> 2 at counter {c0, c1, c2 | (i >> 2) << sh, c3}.
// Random-delivery subsets (Floyd, stream 2, sh = 0) and the event level's
// random /stop schedules (stream 4, sh = 12).
struct DStream {
  uint32_t k0, k1, c0, c1, c2, c3;
  uint4 buf;
  uint32_t widx;
  uint32_t sh;           // block index position in c2: 0 (delivery stream), 12 (crash stream)
  __device__ __forceinline__ uint32_t next() {
    if ((widx & 3u) == 0u) buf = philox4x32_10(k0, k1, make_uint4(c0, c1, c2 | ((widx >> 2) << sh), c3));
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

// One receiver's tally step: acc + popcount(word).  Opaque on purpose (see
// the header comment): the per-receiver count must execute per receiver.
__device__ __forceinline__ uint32_t tally(uint32_t word, uint32_t acc) {
  uint32_t r;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(word), "v"(acc));
  return r;
}

// Same, kept in source order (asm volatile).  For the runtime-W tally loops:
// left free, the scheduler turns the word-major order (G independent ops per
// word) into dependent per-group chains, and the hazard recognizer then puts
// an s_nop between each dependent pair of inline asms it cannot see into.
__device__ __forceinline__ uint32_t tally_ordered(uint32_t word, uint32_t acc) {
  uint32_t r;
  asm volatile("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(word), "v"(acc));
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


// The coin of live node c (compact index) in round r (node.ts:111): bit
// (c & 31) of word (r-1) & 3 of the Philox block
//   ctr = {trial_lo, trial_hi, c >> 5, ((r-1) >> 2) | kStreamCoin << 24},
// i.e. one block holds the coins of 32 nodes for 4 rounds.  coin 1 -> x = 1
// (the reference's Math.random() > 0.5 ? 0 : 1 with P = 1/2).
template <bool WIDE = true>
__device__ __forceinline__ uint4 coin_block(uint32_t k0, uint32_t k1, uint32_t tlo, uint32_t thi, uint32_t c,
                                            uint32_t round) {
  return philox4x32_10<WIDE>(k0, k1, make_uint4(tlo, thi, c >> 5, ((round - 1u) >> 2) | (kStreamCoin << 24)));
}

__device__ __forceinline__ uint32_t coin_word(uint4 b, uint32_t round) {
  const uint32_t j = (round - 1u) & 3u;
  return j == 0u ? b.x : j == 1u ? b.y : j == 2u ? b.z : b.w;
}

// coin_word for a lane-varying round, as three v_bfi_b32 on VGPR masks: the ?:
// chain compiles to v_cndmask_b32 with a VCC / SGPR-pair condition, ~24 cycles
// per wave instruction on gfx950 against ~4 for v_bfi_b32
// (profiles/r03-v7_valu_probe.txt).  The result is a VGPR.
__device__ __forceinline__ uint32_t coin_word_v(uint4 b, uint32_t round) {
  const uint32_t j = (round - 1u) & 3u;
  uint32_t m0 = 0u - (j & 1u), m1 = 0u - (j >> 1);
  asm volatile("" : "+v"(m0), "+v"(m1));
  uint32_t lo, hi, r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(lo) : "v"(m0), "v"(b.y), "v"(b.x));
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(hi) : "v"(m0), "v"(b.w), "v"(b.z));
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m1), "v"(hi), "v"(lo));
  return r;
}

// Random initial values of a network of at most 32 live nodes (one word per
// trial, bit c = compact node c): word t & 3 of the Philox block
// ctr = {q_lo, q_hi, 1 << 31, kStreamInit << 24}, q = t >> 2, so four
// consecutive trials share a block (oracle_random_init, r05).  Networks of
// more than 32 live nodes take words c >> 5 of the trial's own blocks.
constexpr uint32_t kInitShared = 1u << 31;
__device__ __forceinline__ uint4 init_block_small(uint32_t k0, uint32_t k1, uint64_t q) {
  return philox4x32_10<false>(k0, k1, make_uint4((uint32_t)q, (uint32_t)(q >> 32), kInitShared, kStreamInit << 24));
}
__device__ __forceinline__ uint32_t init_word_small(uint32_t k0, uint32_t k1, uint64_t t) {
  return coin_word_v(init_block_small(k0, k1, t >> 2), (uint32_t)(t & 3u) + 1u);
}

// Coins of the tied receivers of one group (lanes = compact nodes 64 g + l).
// The key words are laundered through an empty asm so that Philox's ten round
// keys are not hoisted out of the round loop into permanently live SGPRs.
__device__ __forceinline__ uint64_t coin_ballot(uint32_t k0, uint32_t k1, uint32_t tlo, uint32_t thi,
                                             uint32_t group, uint32_t round, uint64_t tie) {
  const uint32_t lane = threadIdx.x & 63u;
  asm volatile("" : "+s"(k0), "+s"(k1));
  bool c1 = false;
  if ((tie >> lane) & 1ull) {
    // v_mul_lo/hi Philox here: with v_mad_u64_u32's VCC carry-outs the W = 31..32
    // instantiations fail to allocate ("illegal VGPR to SGPR copy")
    const uint4 b = coin_block<false>(k0, k1, tlo, thi, group * 64u + lane, round);
    c1 = (coin_word(b, round) >> (lane & 31u)) & 1u;
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
                                             uint32_t group, uint32_t round, uint64_t tie) {
  const uint2 k = lds_keys(keys);
  tlo = (uint32_t)__builtin_amdgcn_readfirstlane((int)tlo);   // wave-uniform trial id; the asm keeps
  thi = (uint32_t)__builtin_amdgcn_readfirstlane((int)thi);   // Philox's first product on this path
  asm volatile("" : "+s"(tlo), "+s"(thi));
  return coin_ballot(k.x, k.y, tlo, thi, group, round, tie);
}

// The workgroup's LDS histogram added to the launch histogram (one global
// atomic per non-zero bin; call after the __syncthreads that ends the
// counting).  Global atomics on one cache line serialise across the grid, ~12
// ns per workgroup when every workgroup flushes at once
// (tools/atomic_flush_probe.hip, profiles/r03-s2d_atomic_flush_probe.jsonl); the
// round-loop kernels' workgroups end at spread-out times, and 64 histogram
// copies merged by a second kernel measured no faster for them.
__device__ __forceinline__ void flush_hist(const uint32_t *lhist, const KParams &p) {
  for (uint32_t i = threadIdx.x; i < p.hist_len; i += blockDim.x) {
    const uint32_t c = lhist[i];
    if (c) atomicAdd(&p.hist[i], (unsigned long long)c);
  }
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

// Global trial id of launch offset t from the W kernel's parameter block
// ([2,3] trial_begin, [4,5] trial list or 0): trial_begin + t, or in
// trial-list mode trial_begin + list[t] (the matrix-core kernel's deferred
// trials, benor_mfma.h).
__device__ __forceinline__ uint64_t trial_id(const uint32_t *keys, uint32_t t) {
  const uint64_t lp = lds_u64(keys + 4);
  if (lp) t = reinterpret_cast<const uint32_t *>(lp)[t];
  return lds_u64(keys + 2) + t;
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
// "c0 > F" is "c1 < m - F" (no c0 tally exists).  SURE (ODD and m > 2F):
// c1 < m - F or c1 >= m - F > F, so every receiver decides -- 0 if
// c1 < m - F, else 1 -- and one compare per group gives both masks.
// Chain bias g throughout.
template <bool ODD, bool SURE, int W, int K>
__device__ __forceinline__ void decide_k(const uint32_t (&a0)[K][W], const uint32_t (&a1)[K][W], uint32_t m,
                                         uint32_t F, uint64_t tailm, uint64_t (&rest_any)[K], uint64_t (&any0)[K],
                                         uint64_t (&any1)[K]) {
  static_assert(ODD || !SURE, "SURE needs binary votes");
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
      if constexpr (SURE) {
        any0[k] |= d0;
        any1[k] |= vm & ~d0;                                                  // node.ts:102
        asm volatile("" : "+s"(any0[k]), "+s"(any1[k]));
      } else {
        const uint64_t d1 = vcmp_gt(a1[k][g], F + (uint32_t)g) & vm & ~d0;    // node.ts:102
        rest_any[k] |= vm & ~(d0 | d1);
        any0[k] |= d0;
        any1[k] |= d1;
        // fold now: otherwise the ORs sink to the loop exit and all 2W masks stay live
        asm volatile("" : "+s"(rest_any[k]), "+s"(any0[k]), "+s"(any1[k]));
      }
    });
  });
}

}  // namespace benor
