// benor_mfma_small.h -- small networks (2 <= m <= 32 live nodes) on the matrix
// cores: several trials per lane, every receiver's inbox count an e2m1 MFMA
// product.  Instantiated by benor_mfma_small.hip.
//
// Replaces the reference's POST /message round loop (src/nodes/node.ts:43-163)
// for BASELINE configs[1] (N=10, F=4: m = 6) and configs[0]'s shape (N=5,
// F=1: m = 4) -- every lockstep network of at most 32 live nodes that can
// decide (m > F) and has no "?" initial value.
//
// Formulation.  As in benor_mfma.h, a phase's counts are a product
// c[r][t] = sum_s D[r][s] v[s][t] with trials as the N dimension, but a
// network of m <= 32 nodes fills only m of a tile's 32 rows and 64 K.  So a
// lane half h of column t packs S = min(32 / m, 8) trials ("slots") into the
// 32 K positions it supplies, and A is block-diagonal: A[row][k] = 1 iff row
// and k belong to the same slot.  One v_mfma_scale_f32_32x32x64_f8f6f4 pair
// (two 32-row tiles: the 32 rows of each lane half) then counts the inboxes of
// 64 S trials (S = 5 at m = 6: 320 trials, 30 receivers x 30 senders of each
// slot), each receiver's count executed by its own row.
//
// Positions.  Lane (t, h), VGPR v (0..3), nibble n (0..7) is K position
// beta = 4n + 3 - v of half h; slot s owns beta in [s m, s m + m) (node c of
// the slot at s m + c).  x words (bit beta) expand to B nibbles with a shift
// and a mask per VGPR; nibble codes compress back with shifts and masks.
// The accumulator register j of tile T is row (j & 3) + 8 (j >> 2) + 4 h of
// the tile (cdna_hip_programming.md section 3); packed by
// v_cvt_scalef32_pk_fp4_f32 it becomes nibble j & 7 of VGPR 2T + (j >> 3) --
// the position of the receiver as next phase's sender, so A's row slots are
// defined through that position and C -> B is in place (no LDS, no lane move).
//
// A round (node.ts:46-158), per tile T = 0, 1:
//   R-phase: acc = A_T . Bx (A scale 2^3), Bx = +1 for x = 1, -1 for x = 0
//     senders: 8 (c1 - c0); the fp4 conversion saturates it to the proposal
//     +6 (p1), -6 (p0) or 0 ("?", a tie) -- node.ts:63-69.
//   P-phase (node.ts:88-113): from the proposals, three 0/1 operands -- the
//     votes that are not 1, not 0, not "?" -- counted per receiver (zero C):
//     the f32 result is +0.0 iff that count is 0, i.e. the inbox is all 1
//     (n1 = m), all 0 (n0 = m) or all "?" (n0 = n1 = 0); the OR of a slot's
//     rows' bits tests every receiver of the slot at once.
//   In lockstep every receiver's inbox is the whole slot (node.ts:45,171), so
//   it is unanimous: all 1 -> every receiver decides 1 (n1 = m > F,
//   node.ts:102-105), all 0 -> decides 0, all "?" -> every receiver flips its
//   coin (node.ts:110-111) and nobody decides.  Each receiver's row is
//   checked; a slot whose receivers do not all fall in one of the three cases
//   (impossible in lockstep) is re-run with the lane kernel's logic.
// Rounds.  A batch is 64 S trials in the same round.  A slot that halted is
// counted in bin 3r + v.  A tied slot's next x plane is exactly its coins of
// round r (every node took its coin), a pure function of (seed, trial, r), so
// its trial offset goes to the wave's round r + 1 list in LDS and runs there
// with x = coin_word(r) (the continuation idea of benor_mfma.h, here inside one
// launch).  A wave takes a full batch from the deepest full list first, then
// fresh round-1 trials, and drains the partial lists at the end; a trial that
// ties in round kSmallMaxRound (q(m)^3 of them: ~3 % at m = 6) continues
// from there with the lane kernel's per-lane round logic (benor_lane.h), 64
// queued trials at a time; one whose receivers are not unanimous (impossible
// in lockstep) is re-run from round 1 the same way.
#pragma once

#include "benor_lane.h"
#include "benor_mfma.h"

namespace benor {

// small_slots: benor_internal.h

// 32 position bits -> B fragment, e2m1 1.0 (0b0010) where the bit is set:
// VGPR v nibble n <- bit 4n + 3 - v.
__device__ __forceinline__ mf_v4i small_expand(uint32_t w) {
  return mf_v4i{(int)((w >> 2) & 0x22222222u), (int)((w >> 1) & 0x22222222u), (int)(w & 0x22222222u),
                (int)((w << 1) & 0x22222222u)};
}

// (a & m) | (b & ~m) as one v_bfi_b32.  The asm keeps LLVM from turning a
// 0 / ~0 mask back into a select (v_cndmask_b32 with a VCC or SGPR operand,
// ~24 cycles per wave instruction on gfx950: profiles/r03-v7_valu_probe.txt).
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}

// ORs the f32 bits of tile T's accumulator rows into their slots' words:
// register j is receiver position 4 (j & 7) + 3 - (2T + (j >> 3)) (the
// position its packed nibble would take), slot position / MM.
template <int MM>
__device__ __forceinline__ void small_or_rows(const mf_v16f &acc, int T, uint32_t (&o)[small_slots(MM)]) {
  constexpr uint32_t USED = small_slots(MM) * MM;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t beta = 4u * (uint32_t)(j & 7) + 3u - (2u * (uint32_t)T + (uint32_t)(j >> 3));
    if (beta < USED) o[beta / MM] |= __float_as_uint(acc[j]);
  }
#pragma unroll
  for (uint32_t s = 0; s < small_slots(MM); ++s) asm volatile("" : "+v"(o[s]));   // reduce now, free acc
}

// Eight f32 results -> eight e2m1 nibbles (benor_mfma.h pack_fp4_8).
__device__ __forceinline__ uint32_t small_pack(const mf_v16f &acc, int base) { return pack_fp4_8(acc, base); }

// One trial with the lane kernel's per-lane logic (benor_lane.h, KIND 0:
// counts by each receiver's own v_bcnt, coins node.ts:111, k_max), from the
// state after round r0: x plane x1, nobody decided (r0 = 0: /start), coin block
// cw of round group cg (0: none).  Returns the histogram bin; bit 31 flags an
// agreement violation.
template <int MM>
__device__ __forceinline__ uint32_t small_lane_trial(uint32_t k0, uint32_t k1, uint64_t tr, uint32_t x1, uint32_t F, uint32_t k_max,
                                     uint32_t r0, uint4 cw, uint32_t cg) {
  constexpr uint32_t live = MM == 32 ? ~0u : ((1u << MM) - 1u);
  const uint32_t tlo = (uint32_t)tr, thi = (uint32_t)(tr >> 32);
  constexpr uint32_t M = MM, hiT = M >> 1, loT = (M + 1u) >> 1;
  uint32_t dec = 0u, r = r0;
  if (r >= k_max) return x1 == live ? 1u : (x1 == 0u ? 0u : 2u);   // undecided after k_max rounds
  for (;;) {
    ++r;
    uint32_t p0 = 0u, np1 = 0u;
#pragma unroll
    for (int c = MM - 1; c >= 0; --c) {
      const uint32_t s0 = own_count(x1, 0u - loT);                 // c1 - loT: sign = p0 (node.ts:63-69)
      shift_in(p0, s0);
      shift_in(np1, s0 + loT - hiT - 1u);                          // c1 - hiT - 1: sign = not p1
    }
    const uint32_t p1 = ~np1 & live;
    const uint32_t g1 = ((r - 1u) >> 2) + 1u;
    if (2u * (uint32_t)__builtin_popcount(x1) == M && cg != g1) {   // a tie: coins needed (node.ts:110-111)
      cw = coin_block<false>(k0, k1, tlo, thi, 0u, r);     // mul_lo/hi Philox on this divergent path
      cg = g1;
    }
    const uint32_t cwr = coin_word_v(cw, r);
    uint32_t nd0 = 0u, nd1 = 0u, gt1 = 0u, gt0 = 0u;
#pragma unroll
    for (int c = MM - 1; c >= 0; --c) {                           // node.ts:88-113, per receiver
      const uint32_t a = own_count(p0, 0u - (F + 1u)), b = own_count(p1, 0u - (F + 1u));
      shift_in(nd0, a);
      shift_in(nd1, b);
      shift_in(gt1, a - b);
      shift_in(gt0, b - a);
    }
    x1 = nd0 & (~nd1 | gt1 | (~gt0 & cwr)) & live;
    dec |= ~(nd0 & nd1) & live;
    const bool all_dec = dec == live;
    if (all_dec || r >= k_max) {                                   // auto-stop (node.ts:116-145) or k_max
      const uint32_t v = x1 == live ? 1u : (x1 == 0u ? 0u : 2u);
      return (all_dec ? r * 3u + v : v) | ((all_dec && v == 2u) ? 0x80000000u : 0u);
    }
  }
}


// One lane-path trial, counted into the LDS histogram.  A queue entry is a
// trial that tied in every round up to R: its state after round R is x = its
// round-R coins and nobody decided, so the lane kernel's round logic
// continues it from there (coin block of rounds 1-4 in hand, R <= 3); an
// entry with bit 31 set (receivers not unanimous) starts over from round 1.
template <int MM>
__device__ __forceinline__ void small_lane_path(const uint32_t *keys, uint32_t e, uint32_t fixed1, bool random_init, uint32_t F,
                                uint32_t k_max, uint32_t R, uint32_t *lhist, uint32_t hist_len) {
  constexpr uint32_t LIVE = MM == 32 ? ~0u : ((1u << MM) - 1u);
  const uint64_t tr = lds_u64(keys + 2) + (e & 0x7FFFFFFFu);
  const uint2 k2 = lds_keys(keys);
  uint32_t bin;
  if (e >> 31) {
    uint32_t x = fixed1;
    if (random_init) x = init_word_small(k2.x, k2.y, tr) & LIVE;
    bin = small_lane_trial<MM>(k2.x, k2.y, tr, x, F, k_max, 0u, make_uint4(0u, 0u, 0u, 0u), 0u);
  } else {
    const uint4 cw = coin_block<false>(k2.x, k2.y, (uint32_t)tr, (uint32_t)(tr >> 32), 0u, 1u);
    bin = small_lane_trial<MM>(k2.x, k2.y, tr, coin_word(cw, R) & LIVE, F, k_max, R, cw, 1u);
  }
  atomicAdd(&lhist[bin & 0x7FFFFFFFu], 1u);
  if (bin >> 31) atomicAdd(&lhist[hist_len - 1u], 1u);
}

template <int MM>
__global__ void __launch_bounds__(256) benor_mfma_small_kernel(KParams p) {
  constexpr uint32_t S = small_slots(MM);
  constexpr uint32_t BATCH = 64u * S;
  constexpr uint32_t LIVE = MM == 32 ? ~0u : ((1u << MM) - 1u);
  constexpr uint32_t USED = S * MM;                              // position bits in use per lane half
  constexpr uint32_t EMPTY = 0xFFFFFFFFu;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint32_t hist_len = p.hist_len, trial_count = (uint32_t)p.trial_count;
  asm volatile("" : "+s"(hist_len), "+s"(trial_count));
  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint32_t *keys = reinterpret_cast<uint32_t *>(smem + p.hist_bytes - kParamBytes);
  // The wave's LDS slice: the round-2 and round-3 lists (2 BATCH each: a list
  // is drained once it holds a batch, and one batch adds at most BATCH), the
  // round-3 entries' x words (their round-2 coins, carried from the round-2
  // batch that drew their coin block), the lane-path queue (drained 64 at a
  // time) and a fresh batch's init blocks.
  constexpr uint32_t NP = small_init_passes(MM);
  uint32_t *list2 = reinterpret_cast<uint32_t *>(smem + p.hist_bytes) + wv * small_wave_words(MM);
  uint32_t *list3 = list2 + 2u * BATCH, *list3w = list2 + 4u * BATCH, *lq = list2 + 6u * BATCH;
  uint32_t *initw = lq + BATCH + 64u;                     // [NP * 64] uint4 blocks
  for (uint32_t i = threadIdx.x; i < hist_len; i += blockDim.x) lhist[i] = 0u;
  if (threadIdx.x == 0) {
    keys[0] = (uint32_t)p.seed;
    keys[1] = (uint32_t)(p.seed >> 32);
    keys[2] = (uint32_t)p.trial_begin;
    keys[3] = (uint32_t)(p.trial_begin >> 32);
  }
  __syncthreads();

  const bool random_init = p.init_mode == BO_INIT_RANDOM;
  const uint32_t fixed1 = random_init ? 0u : (p.init_plane[0].z & LIVE);
  const uint32_t F = p.F, k_max = p.k_max;
  const uint32_t R = k_max < kSmallMaxRound ? k_max : kSmallMaxRound;   // last matrix-core round

  // Block-diagonal A of the two tiles (see the header): lane (row rho, K half hk).
  mf_v4i A0, A1;
  {
    const uint32_t rho = lane & 31u, hk = lane >> 5, hr = (rho >> 2) & 1u;
    const uint32_t j = (rho & 3u) + 4u * (rho >> 3);
#pragma unroll
    for (int T = 0; T < 2; ++T) {
      const uint32_t vr = 2u * T + (j >> 3), nr = j & 7u;
      const uint32_t br = 4u * nr + 3u - vr;
      const bool row_ok = hk == hr && br < USED;
      const uint32_t sr = br / MM;
      mf_v4i a;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        uint32_t word = 0u;
#pragma unroll
        for (int n = 0; n < 8; ++n) {
          const uint32_t b = 4u * n + 3u - v;
          if (row_ok && b < USED && b / MM == sr) word |= 0x2u << (4 * n);
        }
        a[v] = (int)word;
      }
      if (T == 0) A0 = a;
      else A1 = a;
    }
  }
  const uint32_t used_mask = USED == 32u ? ~0u : ((1u << USED) - 1u);
  const mf_v4i Eu = small_expand(used_mask);
  mf_v16f zero;                                           // the inline constant 0 as every C
#pragma unroll
  for (int j = 0; j < 16; ++j) zero[j] = 0.0f;

  const uint32_t waves_total = gridDim.x * kWavesPerBlock;
  const uint32_t wave_id = blockIdx.x * kWavesPerBlock + wv;
  const uint32_t ngroups = (trial_count + BATCH - 1u) / BATCH;
  uint32_t g = wave_id, len2 = 0u, len3 = 0u, lql = 0u;          // wave-uniform
  uint32_t h0[3] = {0u, 0u, 0u}, h1[3] = {0u, 0u, 0u};             // halts with 0 / 1 in rounds 1..3 (wave totals)
  // diagnostics: [0] start, [1] fresh batches exhausted, [2] lists drained,
  // [3] lane path done, [4] flushed; [5..10] batches: fresh, r2 full, r3 full,
  // r2 partial, r3 partial, lane-path passes
  unsigned long long *tl = p.timeline ? p.timeline + (size_t)wave_id * kTimelineWords : nullptr;
  uint32_t nb[6] = {0u, 0u, 0u, 0u, 0u, 0u};
  bool fresh_done = false;
  if (tl && lane == 0u) tl[0] = (unsigned long long)wall_clock64();

  for (;;) {
    // ---- the next batch: the deepest full list, else fresh round-1 trials
    // (batch g, g + waves_total, ...), else the partial lists
    uint32_t r, n;
    const uint32_t *src = nullptr;
    uint32_t kind;
    if (R >= 3u && len3 >= BATCH) { r = 3u; n = BATCH; len3 -= n; src = list3 + len3; kind = 2u; }
    else if (R >= 2u && len2 >= BATCH) { r = 2u; n = BATCH; len2 -= n; src = list2 + len2; kind = 1u; }
    else if (g < ngroups) { r = 1u; n = trial_count - g * BATCH; n = n < BATCH ? n : BATCH; kind = 0u; }
    else if (len2) { r = 2u; n = len2; src = list2; len2 = 0u; kind = 3u; }
    else if (len3) { r = 3u; n = len3; src = list3; len3 = 0u; kind = 4u; }
    else break;
    if (tl) {
      if (kind >= 3u && !fresh_done && lane == 0u) tl[1] = (unsigned long long)wall_clock64();
      fresh_done = fresh_done || kind >= 3u;
      ++nb[kind];
    }
    r = (uint32_t)__builtin_amdgcn_readfirstlane((int)r);
    n = (uint32_t)__builtin_amdgcn_readfirstlane((int)n);

    // ---- slot s of this lane takes batch entry 64 s + lane; its x word is
    // the initial values (round 1, node.ts:167-188) or, after r - 1 ties, the
    // coins of round r - 1 (node.ts:110-111).
    //   round 1: four consecutive trials share a Philox block of stream 1
    //     (init_word_small): the batch's <= 16 S + 1 blocks are drawn
    //     lane-parallel (NP per lane, chains advanced together) into LDS, block
    //     i at words 4i .. 4i + 3, so entry e's word sits at o + e (o = the
    //     batch's first trial mod 4);
    //   round 2: the slot's coin block of rounds 1-4 (word 0 = round-1 coins),
    //     one per slot, the S chains advanced together; word 1 (round-2 coins)
    //     goes with a trial that ties again to the round-3 list;
    //   round 3: the carried word, no Philox.
    const uint2 kk = lds_keys(keys);
    const uint64_t tb = lds_u64(keys + 2);
    uint32_t toff[S], cw1[S];
    uint32_t w = 0u;
    if (r == 1u) {
      const uint64_t t0 = tb + (uint64_t)g * BATCH;       // the batch's first trial
      const uint32_t o = (uint32_t)t0 & 3u;
      if (random_init) {
        const uint64_t q0 = t0 >> 2;
        uint4 blk[NP];
#pragma unroll
        for (uint32_t i = 0; i < NP; ++i) {
          const uint64_t q = q0 + lane + 64u * i;
          blk[i] = make_uint4((uint32_t)q, (uint32_t)(q >> 32), kInitShared, kStreamInit << 24);
        }
        philox4x32_10_multi<NP>(kk.x, kk.y, blk);
        uint4 *iw4 = reinterpret_cast<uint4 *>(initw);
#pragma unroll
        for (uint32_t i = 0; i < NP; ++i) iw4[lane + 64u * i] = blk[i];
        asm volatile("" ::: "memory");                    // the reads below after every lane's write (in-order LDS)
      }
#pragma unroll
      for (uint32_t s = 0; s < S; ++s) {
        const uint32_t e = s * 64u + lane;
        toff[s] = e < n ? g * BATCH + e : EMPTY;
        const uint32_t x = random_init ? initw[o + e] : fixed1;
        uint32_t keep = (toff[s] >> 31) - 1u;             // ~0 unless the slot is EMPTY
        asm("" : "+v"(keep));                             // a mask, not a select
        w |= (x & LIVE & keep) << (s * MM);
      }
      g += waves_total;
    } else if (r == 2u) {
      uint4 blk[S];
#pragma unroll
      for (uint32_t s = 0; s < S; ++s) {
        const uint32_t e = s * 64u + lane;
        toff[s] = e < n ? src[e] : EMPTY;
        const uint64_t tr = tb + (toff[s] & 0x7FFFFFFFu);
        blk[s] = make_uint4((uint32_t)tr, (uint32_t)(tr >> 32), 0u, kStreamCoin << 24);
      }
      philox4x32_10_multi<S>(kk.x, kk.y, blk);
#pragma unroll
      for (uint32_t s = 0; s < S; ++s) {
        cw1[s] = blk[s].y;
        uint32_t keep = (toff[s] >> 31) - 1u;
        asm("" : "+v"(keep));
        w |= (blk[s].x & LIVE & keep) << (s * MM);
      }
    } else {
      const uint32_t *srcw = list3w + (src - list3);       // the carried words, same index
#pragma unroll
      for (uint32_t s = 0; s < S; ++s) {
        const uint32_t e = s * 64u + lane;
        toff[s] = e < n ? src[e] : EMPTY;
        const uint32_t x = e < n ? srcw[e] : 0u;
        uint32_t keep = (toff[s] >> 31) - 1u;
        asm("" : "+v"(keep));
        w |= (x & LIVE & keep) << (s * MM);
      }
    }
    // B: +1.0 (0x2) where x = 1, -1.0 (0xA) where x = 0, 0 on unused positions
    const mf_v4i Ez = small_expand(used_mask & ~w);
    const mf_v4i Ex = small_expand(w);
    mf_v4i bx;
#pragma unroll
    for (int v = 0; v < 4; ++v) bx[v] = Ex[v] | Ez[v] | (Ez[v] << 2);

    // The products and their folds at raised issue priority (back to 0 for the
    // outcome bookkeeping), so another wave's Philox fills the matrix core's gaps
    // (steady state -1..-5 %, profiles/r04-q_small_setprio_ab.jsonl).
    __builtin_amdgcn_s_setprio(1);
    // ---- R-phase: 8 (c1 - c0) per receiver row -> proposal nibbles (+6 / -6 / 0)
    mf_v4i bp;
    {
      const mf_v16f r0 = mfma_count<3>(A0, bx, zero);
      const mf_v16f r1 = mfma_count<3>(A1, bx, zero);
      bp = mf_v4i{(int)small_pack(r0, 0), (int)small_pack(r0, 8), (int)small_pack(r1, 0), (int)small_pack(r1, 8)};
    }
    // P-phase operands: 1.0 on the used positions whose vote is NOT 1 / NOT 0 /
    // NOT "?" (proposal nibbles: +6 = 0111, -6 = 1111, "?" = 0000).
    mf_v4i bn1, bn0, bnq;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const uint32_t b = (uint32_t)bp[v], b2 = b >> 2;    // bit 1 of a nibble <- its sign bit
      bn1[v] = (int)((b2 | ~b) & (uint32_t)Eu[v]);        // p0 or "?": sign set or bit 1 clear
      bn0[v] = (int)(~b2 & (uint32_t)Eu[v]);              // p1 or "?": sign clear
      bnq[v] = (int)(b & 0x22222222u);                    // p0 or p1: bit 1 set
    }
    // ---- P-phase per tile: a receiver row counts the votes of its slot that
    // are not 1 (n0 + n?), not 0 (n1 + n?), not "?" (n0 + n1).  A count is
    // >= 0, so its f32 is +0.0 exactly when the receiver's inbox is all 1 /
    // all 0 / all "?" (node.ts:92-98), and the OR of the f32 bits of a slot's
    // rows is 0 iff every receiver of the slot saw that.
    uint32_t o1[S], o0[S], oq[S];                         // nonzero: some receiver's count is not 0
#pragma unroll
    for (uint32_t s = 0; s < S; ++s) o1[s] = o0[s] = oq[s] = 0u;
    {
      // all six products first, then their folds: at one wave per SIMD the
      // registers are free and each product's latency hides behind the others
      // (a dependent read of a 32x32x64 result waits ~48 cycles at one wave,
      // tools/mfma32_probe.hip)
      const mf_v16f r10 = mfma_count<3>(A0, bn1, zero), r00 = mfma_count<3>(A0, bn0, zero);
      const mf_v16f rq0 = mfma_count<3>(A0, bnq, zero), r11 = mfma_count<3>(A1, bn1, zero);
      const mf_v16f r01 = mfma_count<3>(A1, bn0, zero), rq1 = mfma_count<3>(A1, bnq, zero);
      small_or_rows<MM>(r10, 0, o1);
      small_or_rows<MM>(r00, 0, o0);
      small_or_rows<MM>(rq0, 0, oq);
      small_or_rows<MM>(r11, 1, o1);
      small_or_rows<MM>(r01, 1, o0);
      small_or_rows<MM>(rq1, 1, oq);
    }

    __builtin_amdgcn_s_setprio(0);
    // ---- per slot: every receiver decided 1 (node.ts:102-105) / decided 0
    // (node.ts:99-101) -> halted in round r (auto-stop, node.ts:116-145); every
    // receiver flipped its coin (node.ts:110-111) -> round r + 1's list, or the
    // lane path after round R; receivers not unanimous (impossible in
    // lockstep) -> the lane path.  (The ORs are < 2^31: 0 - o has bit 31 set
    // iff o != 0.)
    const bool last = r >= R;
    uint32_t *dst = last ? lq : (r == 1u ? list2 : list3);
    uint32_t dlen = last ? lql : (r == 1u ? len2 : len3);
    const bool carry = !last && r == 2u;                  // round-3 entries take their round-2 coins along
    uint32_t c1 = 0u, c0 = 0u, odd_any = 0u;
#pragma unroll
    for (uint32_t s = 0; s < S; ++s) {
      const uint32_t valid = (toff[s] >> 31) ^ 1u;
      const uint32_t n1 = (0u - o1[s]) >> 31, n0 = (0u - o0[s]) >> 31, nq = (0u - oq[s]) >> 31;
      c1 += valid & (n1 ^ 1u);
      c0 += valid & n1 & (n0 ^ 1u);
      const uint32_t tie = valid & n1 & n0 & (nq ^ 1u);
      odd_any |= valid & n1 & n0 & nq;
      const uint64_t bt = ballot(tie != 0u);
      if (tie) {
        const uint32_t at = dlen + __builtin_amdgcn_mbcnt_hi((uint32_t)(bt >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bt, 0u));
        dst[at] = toff[s];
        if (carry) list3w[at] = cw1[s];
      }
      dlen += (uint32_t)__popcll(bt);
    }
    if (last) lql = dlen;
    else if (r == 1u) len2 = dlen;
    else len3 = dlen;
    if (__any(odd_any != 0u)) {                           // impossible in lockstep: queue for the lane path
#pragma unroll
      for (uint32_t s = 0; s < S; ++s) {
        const uint32_t valid = (toff[s] >> 31) ^ 1u;
        const uint32_t odd = valid & ((0u - o1[s]) >> 31) & ((0u - o0[s]) >> 31) & ((0u - oq[s]) >> 31);
        const uint64_t bo = ballot(odd != 0u);
        if (odd)                                          // bit 31: re-run from round 1
          lq[lql + __builtin_amdgcn_mbcnt_hi((uint32_t)(bo >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bo, 0u))] = toff[s] | 0x80000000u;
        lql += (uint32_t)__popcll(bo);
      }
    }
    // wave totals of the halts: bit-sliced ballots (c <= S <= 8)
    uint32_t t1 = 0u, t0 = 0u;
#pragma unroll
    for (uint32_t b = 0; (1u << b) <= S; ++b) {
      t1 += (uint32_t)__popcll(ballot(((c1 >> b) & 1u) != 0u)) << b;
      t0 += (uint32_t)__popcll(ballot(((c0 >> b) & 1u) != 0u)) << b;
    }
    if (r == 1u) { h1[0] += t1; h0[0] += t0; }
    else if (r == 2u) { h1[1] += t1; h0[1] += t0; }
    else { h1[2] += t1; h0[2] += t0; }

    // ---- lane path, 64 queued trials at a time (every lane busy)
    while (lql >= 64u) {
      lql -= 64u;
      small_lane_path<MM>(keys, lq[lql + lane], fixed1, random_init, F, k_max, R, lhist, hist_len);
      if (tl) ++nb[5];
    }
  }
  if (tl && lane == 0u) {
    if (!fresh_done) tl[1] = (unsigned long long)wall_clock64();
    tl[2] = (unsigned long long)wall_clock64();
  }
  // ---- the rest of the lane-path queue
  if (lane < lql) small_lane_path<MM>(keys, lq[lane], fixed1, random_init, F, k_max, R, lhist, hist_len);
  if (tl && lane == 0u) {
    if (lql) ++nb[5];
    tl[3] = (unsigned long long)wall_clock64();
  }
  // halts of the matrix-core rounds: lane 2q + v adds bin 3 (q + 1) + v
  {
    uint32_t c = 0u;
#pragma unroll
    for (uint32_t q = 0; q < 3u; ++q) {
      if (lane == 2u * q) c = h0[q];
      if (lane == 2u * q + 1u) c = h1[q];
    }
    if (lane < 6u && c) atomicAdd(&lhist[3u * (lane / 2u + 1u) + (lane & 1u)], c);
  }
  __syncthreads();
  flush_hist(lhist, p);
  if (tl && lane == 0u) {
    tl[4] = (unsigned long long)wall_clock64();
    for (int i = 0; i < 6; ++i) tl[5 + i] = nb[i];
  }
}

template <int MM>
hipError_t launch_mfma_small_m(const KParams &p, int grid, hipStream_t s) {
  hipLaunchKernelGGL((benor_mfma_small_kernel<MM>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  return hipGetLastError();
}

}  // namespace benor
