// benor_mfma.h -- the matrix-core lockstep kernel: every receiver's inbox
// count as a product on the gfx950 MFMA units.  It runs round 1 of every
// trial; a trial that does not halt there is handed to the popcount W kernel
// (trial-list mode), which re-runs it from round 1.
//
// Formulation.  In one phase, receiver r of trial t counts the votes of the
// senders it hears: c[r][t] = sum_s D[r][s] * v[s][t], D the delivery matrix
// (lockstep: every live sender reaches every live receiver, node.ts:45,171),
// v the 0/1 vote plane.  With the trials of a wave as the N dimension this is
// a (receivers x senders) . (senders x 32 trials) product, which
// v_mfma_scale_f32_32x32x64_f8f6f4 computes on e2m1 (fp4) operands: 0 and 1
// are exact e2m1 values, and the f32 accumulation of at most 4096 unit
// products is exact, so every count -- and every decision -- is bit-identical
// to the popcount kernels and the oracle.  One instruction does 32 x 32 x 64 =
// 65536 receiver-sender terms; tools/mfma_probe.hip measured it at 16.1 ns per
// SIMD under full load, 3.5x the v_bcnt_u32_b32 rate in terms per second.
//
// Eligible shapes (plan_geometry, variant 7): lockstep, 64 < m <= 1024, m > F
// (decisions possible).  KIND (KParams::G):
//  0 "sure": every vote count odd (m odd, an even number of "?" initial
//    values) and m > 2F.  No R-phase count ties (no "?" proposal) and every
//    receiver decides in the P-phase (decide_k's SURE case), so every trial
//    halts in round 1 with x = the decided value.  The headline N=1024/F=341
//    and configs[2] N=256/F=85.
//  1 m > 2F, ties possible (even vote count): a trial halts in round 1 unless
//    some receiver proposed "?" (node.ts:63-69) -- then it is deferred.
//  2 F < m <= 2F: a receiver decides only when one value has more than F
//    votes; a trial with a "?" proposal or an undecided receiver is deferred.
// Deferred trials (their offsets within the launch) are appended to
// p.defer_list; the host runs them through the W kernel in trial-list mode
// right after, on the same stream, so every trial is counted exactly once.
// The network API's single-trial launch (per-node state) stays on the W kernel.
//
// Layout (one wave = one tile of 32 trials, trial t0 + (lane & 31)):
//  * B operand, R-phase: K chunk c holds senders 64c .. 64c+63; lane half
//    h = lane >> 5 brings 32 of them (x-plane word 2c + h) as 32 e2m1 nibbles
//    in 4 VGPRs (nibble i of VGPR v = sender bit 4i + v, value 1.0 = 0b0010).
//  * A operand: all ones (e2m1 1.0): D restricted to live nodes.  The 32-row
//    receiver tiles are identical products; an empty asm on A per tile keeps
//    the compiler from merging them -- each receiver's count is executed.
//  * C/D: accumulator register j of lane l is receiver row
//    (j & 3) + 8 (j >> 2) + 4 (l >> 5) of the tile, trial column l & 31
//    (cdna_hip_programming.md section 3) -- the same column as the B operand,
//    so a tile's 16 results per lane become the next phase's B operand in
//    place: no LDS, no lane exchange.
//  * R-phase: A carries scale 2^4, C = -8M (M binary votes), so the result is
//    8 (c1 - c0) (node.ts:63-69): positive for p1, negative for p0, zero for a
//    tie ("?").  v_cvt_scalef32_pk_fp4_f32 packs two results per byte and
//    saturates: the proposal plane is +6 / -6 / 0 nibbles, the next product's
//    B operand in place.
//  * P-phase: S = sum of proposals = 6 (n1 - n0); with no "?" among them
//    n0 + n1 = m, so thresholds on S are thresholds on c0 = n0 and c1 = n1
//    (node.ts:99-105), again carried by C.
//  * Padding: senders >= m are zero bits in the x words; receiver rows >= m in
//    the last tile are masked out of the P-phase operand and start their
//    P-phase accumulator at NaN, which the min / max reductions skip.
#pragma once

#include "benor_device.h"

namespace benor {

typedef int mf_v4i __attribute__((ext_vector_type(4)));
typedef int mf_v8i __attribute__((ext_vector_type(8)));
typedef float mf_v16f __attribute__((ext_vector_type(16)));

// 32 receivers x 32 trials x 64 senders, e2m1 operands; A scaled by 2^SA
// (E8M0 127 + SA), B unit scale.
template <int SA = 0>
__device__ __forceinline__ mf_v16f mfma_count(mf_v4i a, mf_v4i b, mf_v16f c) {
  const mf_v8i a8 = __builtin_shufflevector(a, a, 0, 1, 2, 3, -1, -1, -1, -1);   // fp4 reads the low 4 VGPRs
  const mf_v8i b8 = __builtin_shufflevector(b, b, 0, 1, 2, 3, -1, -1, -1, -1);
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, 127 + SA, 0, 127);
}

// Sign bits of four f32 results as bytes (0xff where negative): v_perm_b32
// selector 9 / 11 replicate bit 31 of the low / high source, 12 gives 0x00.
__device__ __forceinline__ uint32_t sign_bytes(float e0, float e1, float e2, float e3) {
  const uint32_t lo = __builtin_amdgcn_perm(__float_as_uint(e1), __float_as_uint(e0), 0x0C0C0B09u);
  const uint32_t hi = __builtin_amdgcn_perm(__float_as_uint(e3), __float_as_uint(e2), 0x0B090C0Cu);
  return lo | hi;
}

// Eight results -> eight e2m1 nibbles, 1.0 where the result is negative:
// results 0..3 in the low nibbles of bytes 0..3, results 4..7 in the high ones.
__device__ __forceinline__ uint32_t pack_signs8(const mf_v16f &acc, int base) {
  const uint32_t s0 = sign_bytes(acc[base + 0], acc[base + 1], acc[base + 2], acc[base + 3]);
  const uint32_t s1 = sign_bytes(acc[base + 4], acc[base + 5], acc[base + 6], acc[base + 7]);
  return (s0 & 0x02020202u) | (s1 & 0x20202020u);
}

// Eight results -> eight e2m1 nibbles: v_cvt_scalef32_pk_fp4_f32 rounds two
// f32 into byte k (src0 in bits 8k..8k+3, src1 in 8k+4..8k+7) and saturates:
// every R-phase result has |value| >= 8 (the count is scaled by 16 through
// the MFMA's A scale and the threshold sits half a vote from it), so each
// nibble is exactly +6.0 (0x7, proposal 1) or -6.0 (0xF, proposal 0).
__device__ __forceinline__ uint32_t pack_fp4_8(const mf_v16f &acc, int base) {
  uint32_t r;
  asm volatile("" : "=v"(r));   // no initial value: the four conversions write every byte (no v_mov 0)
  r = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(r, acc[base + 0], acc[base + 1], 1.0f, 0);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(r, acc[base + 2], acc[base + 3], 1.0f, 1);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(r, acc[base + 4], acc[base + 5], 1.0f, 2);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(r, acc[base + 6], acc[base + 7], 1.0f, 3);
  return r;
}

// h ? a : b for a lane-half flag, as one v_bfi_b32 on the 0 / ~0 VGPR mask hm:
// a lane-varying ?: compiles to v_cndmask_b32 with an SGPR-pair mask, ~24 cycles
// per wave instruction on gfx950 against ~4 for v_bfi_b32
// (profiles/r03-v7_valu_probe.txt).
__device__ __forceinline__ uint32_t half_sel(uint32_t hm, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(hm), "v"(a), "v"(b));
  return r;
}

// x1 words of chunks 4j .. 4j+3 of this lane half h from its /start Philox
// block r (block 2j + h): half h keeps words h and 2 + h and trades the other
// two with lane l ^ 32 (ds_bpermute).
__device__ __forceinline__ void half_trade(const uint4 &r, uint32_t h, uint32_t (&xw)[4]) {
  uint32_t hm = 0u - h;
  asm volatile("" : "+v"(hm));                   // a VGPR mask, not a select condition
  const uint32_t keep_a = half_sel(hm, r.y, r.x), keep_b = half_sel(hm, r.w, r.z);
  const uint32_t give_a = half_sel(hm, r.x, r.y), give_b = half_sel(hm, r.z, r.w);
  const int xa = (int)(((threadIdx.x & 63u) ^ 32u) << 2);   // lane l ^ 32 (no __shfl_xor bounds select)
  const uint32_t recv_a = (uint32_t)__builtin_amdgcn_ds_bpermute(xa, (int)give_a);
  const uint32_t recv_b = (uint32_t)__builtin_amdgcn_ds_bpermute(xa, (int)give_b);
  xw[0] = half_sel(hm, recv_a, keep_a);
  xw[1] = half_sel(hm, recv_b, keep_b);
  xw[2] = half_sel(hm, keep_a, recv_a);
  xw[3] = half_sel(hm, keep_b, recv_b);
}

// 32 sender bits -> the 4 VGPRs of one lane's B fragment (nibble i of VGPR v
// = bit 4i + v of the word, as e2m1 1.0).
__device__ __forceinline__ mf_v4i expand_votes(uint32_t w) {
  return mf_v4i{(int)((w << 1) & 0x22222222u), (int)(w & 0x22222222u), (int)((w >> 1) & 0x22222222u),
                (int)((w >> 2) & 0x22222222u)};
}

template <int W, bool HALF, int KIND>
__global__ void __launch_bounds__(256) benor_mfma_kernel(KParams p) {
  constexpr int MT = 2 * W - (HALF ? 1 : 0);   // 32-receiver tiles (HALF: the last chunk holds <= 32 senders)
  constexpr int KP = (MT + 1) / 2;             // P-phase K chunks: two tiles' results each
  constexpr int NB = (W + 1) / 2;              // Philox init blocks per trial (128 senders each)
  constexpr int NJ = (NB + 1) / 2;             // blocks per lane: half h draws blocks h, h + 2, ...
  constexpr bool SURE = KIND == 0;
  // (r05 measured the SURE W <= 4 proposal packing and P-phase fold through
  // v_cvt_scalef32_pk_fp4_f32 instead of v_perm sign bytes and the f32 sign
  // fold: 10 % fewer VALU, 8-12 % slower at configs[2] -- the conversion is
  // the slower instruction; profiles/r05-h_mfma_fp4_fold_ab.jsonl.  And one
  // bias accumulator for both phases where they coincide (N = 3F + 1: 16 VGPRs
  // fewer, 5 waves per SIMD at W = 3): configs[2] and the headline unchanged
  // within 1 %, with or without a grid sized to the resident waves (that one
  // 2-5 % slower); profiles/r05-k_eqb_resident_grid_ab.jsonl, r05-l_mfma_eqb_ab.jsonl.
  // Nor did distinct product-phase priorities per wave slot (s_setprio 1..3 by
  // HW_ID, so that one wave's products run ahead of the others'): within
  // noise everywhere; profiles/r05-o_mfma_slot_priority_ab.jsonl.)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u, h = lane >> 5;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  // Continuation pass (KIND > 0): round `cont` of the listed trials, every one
  // of which tied in rounds 1 .. cont-1 -- all proposals "?", all votes "?",
  // so every receiver took its coin (node.ts:63-69, 110-111) and the x plane
  // of round cont is the coins of round cont-1.
  const uint32_t cont = SURE ? 0u : p.cont_round;
  uint32_t m = p.m, hist_len = p.hist_len;
  uint32_t trial_count = cont ? *p.trial_list_len : (uint32_t)p.trial_count;
  asm volatile("" : "+s"(m), "+s"(hist_len), "+s"(trial_count));

  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint32_t *keys = reinterpret_cast<uint32_t *>(smem + p.hist_bytes - kParamBytes);   // as the W kernel
  for (uint32_t i = threadIdx.x; i < hist_len; i += blockDim.x) lhist[i] = 0u;
  if (threadIdx.x == 0) {
    keys[0] = (uint32_t)p.seed;
    keys[1] = (uint32_t)(p.seed >> 32);
    keys[2] = (uint32_t)p.trial_begin;
    keys[3] = (uint32_t)(p.trial_begin >> 32);
  }
  __syncthreads();

  const bool random_init = p.init_mode == BO_INIT_RANDOM;
  const uint32_t M1 = cont ? m : m - p.init_q;  // binary votes ("?" inputs excluded in round 1)
  // KIND 0: every vote count odd, so p0 = (c1 <= M1 >> 1) is the sign of
  //   c1 - (M1 >> 1) - 0.5 (node.ts:63-69), packed by v_perm as a 0/1 plane
  //   (e2m1 1.0 = p0); in the P-phase the sign of c0 - F - 0.5 is "not d0"
  //   = x1 (node.ts:99-105: every receiver decides, m > 2F).
  // KIND 1, 2: the count enters scaled by 16 (A scale 2^4) against C = -8 M1,
  //   so acc = 8 (c1 - c0): >= 8 for p1, <= -8 for p0, 0 for "?"; the fp4
  //   conversion saturates it to +6 / -6 and keeps 0.  The P-phase sum is
  //   S = 6 (n1 - n0), and where no proposal is "?", n0 + n1 = m:
  //   KIND 1 (m > 2F): acc = S - 6 (m - 2F) + 3 = 12 (F - c0) + 3, negative
  //     exactly when c0 > F (decide 0, node.ts:99-101), else c1 >= m - F > F
  //     (decide 1, node.ts:102-105);
  //   KIND 2 (F < m <= 2F): acc = S = 6 (c1 - c0); the receiver decides iff
  //     |c1 - c0| > 2F - m (c0 > F or c1 > F), for the value of the sign.
  const float bias_r = SURE ? -((float)(M1 >> 1) + 0.5f) : -8.0f * (float)M1;
  const float bias_p = SURE ? -((float)p.F + 0.5f) : (KIND == 2 ? 0.0f : 3.0f - 6.0f * (float)(m - 2u * p.F));
  const float dec_thr = 6.0f * (float)(2u * p.F - m) + 3.0f;   // KIND 2: |acc| > dec_thr <=> decided
  mf_v16f cr, cp, cp_tail;
  // Receiver rows of the last tile that exist: nibble masks for its packed
  // R-phase results; KIND 1, 2 start their P-phase results from NaN where no
  // receiver exists, which v_min3_f32 / v_max3_f32 skip (IEEE minNum /
  // maxNum).  KIND 0 needs no mask there (see the P-phase).
  const uint32_t mrem = m - 32u * (uint32_t)(MT - 1);   // 1..32
  uint32_t tail0 = 0, tail1 = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t row = (uint32_t)((j & 3) + 8 * (j >> 2)) + 4u * h;
    const bool live = row < mrem;
    cr[j] = bias_r;
    cp[j] = bias_p;
    cp_tail[j] = live ? bias_p : __builtin_nanf("");
    const uint32_t nib = !live ? 0u : SURE ? ((j & 4) ? 0x20u : 0x02u) << (8 * (j & 3)) : 0xFu << (4 * (j & 7));
    if (j < 8) tail0 |= nib;
    else tail1 |= nib;
  }
  // Fixed initial values: the same x1 words for every trial.
  uint32_t fixed_w[W];
  if (!random_init) {
#pragma unroll
    for (int c = 0; c < W; ++c) {
      const uint4 q = p.init_plane[c];
      fixed_w[c] = h ? q.w : q.z;
    }
  }
  // Valid sender bits of this lane's word in the last chunk (word 2(W-1) + h).
  const int last_bits = (int)m - 32 * (2 * (W - 1) + (int)h);
  const uint32_t last_mask = last_bits >= 32 ? ~0u : (last_bits <= 0 ? 0u : ((1u << last_bits) - 1u));

  mf_v4i ones = {0x22222222, 0x22222222, 0x22222222, 0x22222222};
  uint32_t f_all = 0, f_1 = 0, f_2 = 0;   // halts, halts with some x = 1, with both values
  const uint32_t ngroups = (trial_count + 31u) >> 5;
  const uint32_t waves_total = gridDim.x * kWavesPerBlock;
  const uint32_t wave_id = blockIdx.x * kWavesPerBlock + wv;
  // KIND > 0: this wave's deferred trials go to its own segment of
  // p.defer_seg (no contended atomics in the loop), copied to the compact
  // list p.defer_list at the end with one atomic per wave.
  uint32_t n_def = 0;
  uint32_t *seg = SURE ? nullptr : p.defer_seg + (size_t)wave_id * p.defer_seg_cap;
  for (uint32_t g = wave_id; g < ngroups; g += waves_total) {
    const uint32_t t = (g << 5) + (lane & 31u);
    const bool valid = t < trial_count;
    const uint32_t toff = cont ? (valid ? p.trial_list[t] : 0u) : t;   // the trial's offset in the launch
    // ---- /start (node.ts:167-188): this lane's x1 words 2c + h, c < W.
    uint32_t xw[W];
    if (SURE ? false : cont != 0u) {
      // coins of round cont-1: word (cont-2) & 3 of the block (trial, node
      // group 2c + h, round group (cont-2) >> 2) of the coin stream (coin_block)
      const uint64_t trial = lds_u64(keys + 2) + toff;
      const uint2 kk = lds_keys(keys);
#pragma unroll
      for (int c = 0; c < W; ++c) {
        const uint4 r = coin_block(kk.x, kk.y, (uint32_t)trial, (uint32_t)(trial >> 32), 32u * (2u * c + h), cont - 1u);
        xw[c] = coin_word(r, cont - 1u);
      }
    } else if (random_init) {
      const uint64_t trial = lds_u64(keys + 2) + t;
      const uint2 kk = lds_keys(keys);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        // Block b = 2j + h: words 4b .. 4b+3 = chunks 2b, 2b+1.  Half h keeps
        // words 4b + h, 4b + 2 + h and trades the other two with lane l ^ 32.
        const uint4 r = philox4x32_10(kk.x, kk.y,
                                      make_uint4((uint32_t)trial, (uint32_t)(trial >> 32), 2u * j + h, kStreamInit << 24));
        uint32_t q4[4];
        half_trade(r, h, q4);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (4 * j + q < W) xw[4 * j + q] = q4[q];
      }
    } else {
#pragma unroll
      for (int c = 0; c < W; ++c) xw[c] = fixed_w[c];
    }
    xw[W - 1] &= last_mask;
    mf_v4i bx[W];
#pragma unroll
    for (int c = 0; c < W; ++c) bx[c] = expand_votes(xw[c]);

    // ---- R-phase ("proposal phase", node.ts:46-82): every receiver tile
    // counts the x plane; the packed result is its proposal.
    uint32_t bp[MT][2];
    uint32_t qz = 0u;                          // KIND > 0: a live receiver proposed "?"
    if constexpr (SURE && W <= 4) {
      // Few products per tile (W): the sign packing of tile i - 1 is issued
      // among tile i's products, a few VALU per MFMA, so it runs in their
      // shadow (two accumulators live).  The wave raises its issue priority for
      // the two product phases (back to 0 after the P-phase fold), so another
      // wave's Philox / expansion VALU fills the matrix core's gaps rather than
      // delaying its products: configs[2] -3 % (profiles/r04-o_setprio_ab.jsonl).
      __builtin_amdgcn_s_setprio(1);
      mf_v16f racc[2];
#pragma unroll
      for (int i = 0; i <= MT; ++i) {
        if (i < MT) {
          asm volatile("" : "+v"(ones));
          mf_v16f acc = mfma_count(ones, bx[0], cr);
#pragma unroll
          for (int c = 1; c < W; ++c) acc = mfma_count(ones, bx[c], acc);
          racc[i & 1] = acc;
        }
        if (i > 0) {
          bp[i - 1][0] = pack_signs8(racc[(i - 1) & 1], 0);
          bp[i - 1][1] = pack_signs8(racc[(i - 1) & 1], 8);
        }
        if (i < MT && i > 0) {
#pragma unroll
          for (int c = 0; c < W; ++c) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, (16 + W - 1) / W, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      asm volatile("" : "+v"(ones));
      if constexpr (SURE) {
        mf_v16f acc = mfma_count(ones, bx[0], cr);
#pragma unroll
        for (int c = 1; c < W; ++c) acc = mfma_count(ones, bx[c], acc);
        bp[i][0] = pack_signs8(acc, 0);
        bp[i][1] = pack_signs8(acc, 8);
      } else {
        mf_v16f acc = mfma_count<4>(ones, bx[0], cr);
#pragma unroll
        for (int c = 1; c < W; ++c) acc = mfma_count<4>(ones, bx[c], acc);
        bp[i][0] = pack_fp4_8(acc, 0);
        bp[i][1] = pack_fp4_8(acc, 8);
        // a "?" nibble is 0: bit 1 clear (+6 = 0x7, -6 = 0xF)
        const uint32_t l0 = i == MT - 1 ? (tail0 & 0x22222222u) : 0x22222222u;
        const uint32_t l1 = i == MT - 1 ? (tail1 & 0x22222222u) : 0x22222222u;
        qz |= (~bp[i][0] & l0) | (~bp[i][1] & l1);
      }
      __builtin_amdgcn_sched_barrier(0);   // one tile's accumulator live at a time
    }
    bp[MT - 1][0] &= tail0;
    bp[MT - 1][1] &= tail1;
    mf_v4i pb[KP];
#pragma unroll
    for (int c = 0; c < KP; ++c)
      pb[c] = mf_v4i{(int)bp[2 * c][0], (int)bp[2 * c][1], 2 * c + 1 < MT ? (int)bp[2 * c + 1][0] : 0,
                     2 * c + 1 < MT ? (int)bp[2 * c + 1][1] : 0};

    // ---- P-phase ("voting phase", node.ts:83-158): every receiver tile
    // counts the proposals; the sign of its result is its decision.  The
    // outcome needs, per trial, whether some receiver decided 0 and whether
    // some decided 1 (and for KIND 2 whether every receiver decided).
    uint32_t any1, any0, halt = (uint32_t)ballot(valid);
    if constexpr (SURE) {
      uint32_t s_or = 0u, s_and = ~0u;        // sign bit = "not d0" = x1
      if constexpr (W <= 4) {
        // tile i - 1's sign fold among tile i's products, as the R-phase
        mf_v16f pacc[2];
#pragma unroll
        for (int i = 0; i <= MT; ++i) {
          if (i < MT) {
            asm volatile("" : "+v"(ones));
            mf_v16f acc = mfma_count(ones, pb[0], cp);
#pragma unroll
            for (int c = 1; c < KP; ++c) acc = mfma_count(ones, pb[c], acc);
            pacc[i & 1] = acc;
          }
          if (i > 0) {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
              const uint32_t u = __float_as_uint(pacc[(i - 1) & 1][j]);
              s_or |= u;
              s_and &= u;
            }
          }
          if (i < MT && i > 0) {
#pragma unroll
            for (int c = 0; c < KP; ++c) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, (16 + KP - 1) / KP, 0);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_s_setprio(0);
      } else
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        asm volatile("" : "+v"(ones));
        mf_v16f acc = mfma_count(ones, pb[0], cp);
#pragma unroll
        for (int c = 1; c < KP; ++c) acc = mfma_count(ones, pb[c], acc);
        // Padded receiver rows of the last tile need no mask here: A is all
        // ones on every row and C is the same bias, so a padded row computes
        // exactly the count of the live rows of its trial column (the padded
        // senders are masked out of the operand).  Folding it in changes
        // neither the OR nor the AND of the sign bits (r02: N=256 +6 %).
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const uint32_t u = __float_as_uint(acc[j]);
          s_or |= u;
          s_and &= u;
        }
        asm volatile("" : "+v"(s_or), "+v"(s_and));   // fold tile by tile: one accumulator live
        __builtin_amdgcn_sched_barrier(0);
      }
      const uint64_t b1 = ballot(s_or >> 31);          // some receiver decided 1
      const uint64_t b0 = ballot(!(s_and >> 31));      // some receiver decided 0
      any1 = (uint32_t)b1 | (uint32_t)(b1 >> 32);
      any0 = (uint32_t)b0 | (uint32_t)(b0 >> 32);
    } else {
      float mn = __builtin_inff(), mx = -__builtin_inff(), ma = __builtin_inff();
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        asm volatile("" : "+v"(ones));
        mf_v16f acc = mfma_count(ones, pb[0], i < MT - 1 ? cp : cp_tail);
#pragma unroll
        for (int c = 1; c < KP; ++c) acc = mfma_count(ones, pb[c], acc);
#pragma unroll
        for (int j = 0; j < 16; j += 2) {
          mn = fminf(fminf(mn, acc[j]), acc[j + 1]);
          mx = fmaxf(fmaxf(mx, acc[j]), acc[j + 1]);
          if constexpr (KIND == 2) ma = fminf(fminf(ma, __builtin_fabsf(acc[j])), __builtin_fabsf(acc[j + 1]));
        }
        asm volatile("" : "+v"(mn), "+v"(mx), "+v"(ma));   // fold tile by tile: one accumulator live
        __builtin_amdgcn_sched_barrier(0);
      }
      // ---- columns with a "?" proposal or an undecided receiver are deferred
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
      const uint64_t b1 = ballot(mx > 0.0f);            // some receiver decided 1
      const uint64_t b0 = ballot(mn < 0.0f);            // some receiver decided 0
      any1 = (uint32_t)b1 | (uint32_t)(b1 >> 32);
      any0 = (uint32_t)b0 | (uint32_t)(b0 >> 32);
    }
    // ---- outcome: bins 3R + v, per trial column (lanes n, n + 32)
    any1 &= halt;
    any0 &= halt;
    f_all += (uint32_t)__builtin_popcount(halt);
    f_1 += (uint32_t)__builtin_popcount(any1);
    f_2 += (uint32_t)__builtin_popcount(any1 & any0);
  }
  if constexpr (!SURE) {
    // The waves' deferred trials -> the compact list, one global atomic per
    // workgroup: atomics on one counter serialise across the grid (~12 ns
    // each, tools/atomic_flush_probe.hip), and one per wave held KIND 1
    // shapes back (N=256 F=0 -26 % at 8 workgroups per CU against 2;
    // profiles/r03-s2n_mfma_blocks_per_cu_inproc.jsonl).  Parameter-block words
    // 4..7 hold the waves' counts, then the workgroup's base.
    if (n_def > p.defer_seg_cap) {   // segment overflow: the extra trials are dropped and the launch flagged
      if (lane == 0) atomicOr(p.overflow, 1u);
      n_def = p.defer_seg_cap;
    }
    uint32_t *wdef = keys + 4;
    if (lane == 0) wdef[wv] = n_def;
    __syncthreads();
    uint32_t before = 0u, total = 0u;
#pragma unroll
    for (uint32_t w = 0; w < (uint32_t)kWavesPerBlock; ++w) {
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

  // outcome bins 3R + v of the halting round R (1, or the continuation's round)
  const uint32_t rb = 3u * (cont ? cont : 1u);
  const uint32_t hc = lane == rb ? f_all - f_1 : (lane == rb + 1u ? f_1 - f_2 : (lane == rb + 2u ? f_2 : 0u));
  if (hc) atomicAdd(&lhist[lane], hc);
  if (lane == 0 && f_2) atomicAdd(&lhist[hist_len - 1u], f_2);                   // disagreement counter
  __syncthreads();
  flush_hist(lhist, p);
}

template <int W, int KIND>
static inline void launch_mfma_kind(const KParams &p, int grid, hipStream_t s) {
  if (p.m <= 64u * (uint32_t)(W - 1) + 32u)
    hipLaunchKernelGGL((benor_mfma_kernel<W, true, KIND>), dim3(grid), dim3(64 * kWavesPerBlock), p.hist_bytes, s, p);
  else
    hipLaunchKernelGGL((benor_mfma_kernel<W, false, KIND>), dim3(grid), dim3(64 * kWavesPerBlock), p.hist_bytes, s, p);
}

template <int W>
hipError_t launch_mfma(const KParams &p, int grid, hipStream_t s) {
  if (p.G == 0u) launch_mfma_kind<W, 0>(p, grid, s);
  else if (p.G == 1u) launch_mfma_kind<W, 1>(p, grid, s);
  else launch_mfma_kind<W, 2>(p, grid, s);
  return hipGetLastError();
}

}  // namespace benor
