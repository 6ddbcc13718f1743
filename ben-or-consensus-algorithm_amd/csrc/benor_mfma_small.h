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
// and a mask per VGPR; sign nibbles compress back with three bit-field inserts.
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
//   P-phase (node.ts:88-113): with Bp the proposals, |Bp| and -Bp,
//     U = A.Bp + A.|Bp| - (12m - 6) = 12 n1 - 12m + 6 > 0  iff  n1 = m,
//     V = A.(-Bp) + A.|Bp| - (12m - 6) = 12 n0 - 12m + 6 > 0  iff  n0 = m,
//     W = 4 - A.|Bp| = 4 - 6 (n0 + n1) > 0  iff  every vote is "?".
//   In lockstep every receiver's inbox is the whole slot (node.ts:45,171), so
//   it is unanimous: all 1 -> every receiver decides 1 (n1 = m > F,
//   node.ts:102-105), all 0 -> decides 0, all "?" -> every receiver flips its
//   coin (node.ts:110-111) and nobody decides.  Each receiver's sign bits are
//   checked; a slot whose receivers do not all fall in one of the three cases
//   (impossible in lockstep) is re-run by the lane path below, as is a trial
//   that ties kSmallMaxRound times.
// A slot that decided is counted in bin 3r + v.  A tied slot's next x plane
// is exactly its coins of round r (every node took its coin), a pure function
// of (seed, trial, r): it is queued, as a trial offset, on the wave's round
// r + 1 list in LDS, and runs there with x = coin_word(r) (the continuation
// idea of benor_mfma.h, here inside one persistent launch).  A wave takes a
// full batch from the deepest full list first, then fresh round-1 trials, and
// drains the partial lists at the end.
//
// Lane path: a trial is re-run from round 1 with the lane kernel's per-lane
// round logic (benor_lane.h, KIND 0), one trial per lane, 64 queued trials at
// a time (q(m)^3 of the trials: ~3 % at m = 6).
#pragma once

#include "benor_lane.h"
#include "benor_mfma.h"

namespace benor {

constexpr uint32_t kSmallMaxRound = 3;   // rounds on the matrix cores; a later tie -> lane path

// small_slots / small_wave_words: benor_internal.h

// 32 position bits -> B fragment, e2m1 1.0 (0b0010) where the bit is set:
// VGPR v nibble n <- bit 4n + 3 - v.
__device__ __forceinline__ mf_v4i small_expand(uint32_t w) {
  return mf_v4i{(int)((w >> 2) & 0x22222222u), (int)((w >> 1) & 0x22222222u), (int)(w & 0x22222222u),
                (int)((w << 1) & 0x22222222u)};
}

// Sign bits (bit 3 of every nibble) of a fragment -> position bits
// (bit 4n + 3 - v <- bit 3 of VGPR v nibble n).
__device__ __forceinline__ uint32_t small_compress(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3) {
  const uint32_t t01 = (v0 & 0x88888888u) | ((v1 >> 1) & 0x44444444u);
  const uint32_t t23 = (v2 & 0x88888888u) | ((v3 >> 1) & 0x44444444u);
  return t01 | (t23 >> 2);
}

// Eight f32 results -> eight e2m1 nibbles (benor_mfma.h pack_fp4_8).
__device__ __forceinline__ uint32_t small_pack(const mf_v16f &acc, int base) { return pack_fp4_8(acc, base); }

// One trial from round 1 with the lane kernel's per-lane logic (benor_lane.h,
// KIND 0: counts by each receiver's own v_bcnt, coins node.ts:111, k_max).
// Returns the histogram bin; bit 31 flags an agreement violation.
template <int MM>
__device__ uint32_t small_lane_trial(uint32_t k0, uint32_t k1, uint64_t tr, uint32_t x1, uint32_t F, uint32_t k_max) {
  constexpr uint32_t live = MM == 32 ? ~0u : ((1u << MM) - 1u);
  const uint32_t tlo = (uint32_t)tr, thi = (uint32_t)(tr >> 32);
  constexpr uint32_t M = MM, hiT = M >> 1, loT = (M + 1u) >> 1;
  uint32_t dec = 0u, r = 0u, cg = 0u;
  uint4 cw = make_uint4(0u, 0u, 0u, 0u);
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
      uint32_t kk0 = k0, kk1 = k1;
      asm volatile("" : "+s"(kk0), "+s"(kk1));
      cw = coin_block(kk0, kk1, tlo, thi, 0u, r);
      cg = g1;
    }
    const uint32_t cwr = coin_word(cw, r);
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

template <int MM>
__global__ void __launch_bounds__(256) benor_mfma_small_kernel(KParams p) {
  constexpr uint32_t S = small_slots(MM);
  constexpr uint32_t BATCH = 64u * S;
  constexpr uint32_t LIVE = MM == 32 ? ~0u : ((1u << MM) - 1u);
  constexpr uint32_t USED = S * MM;                              // position bits in use per lane half
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint32_t hist_len = p.hist_len, trial_count = (uint32_t)p.trial_count;
  asm volatile("" : "+s"(hist_len), "+s"(trial_count));
  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint32_t *keys = reinterpret_cast<uint32_t *>(smem + p.hist_bytes - kParamBytes);
  uint32_t *wbase = reinterpret_cast<uint32_t *>(smem + p.hist_bytes) + wv * small_wave_words(MM);
  uint32_t *list2 = wbase, *list3 = wbase + 2u * BATCH, *lq = wbase + 4u * BATCH;   // lq: lane-path queue
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
  // Valid position bits and their -1 nibbles' base (every used position +-1).
  const uint32_t used_mask = USED == 32u ? ~0u : ((1u << USED) - 1u);
  mf_v16f cbig, zero;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    cbig[j] = -(12.0f * (float)MM - 6.0f);
    zero[j] = 0.0f;
  }
  mf_v16f four;
#pragma unroll
  for (int j = 0; j < 16; ++j) four[j] = 4.0f;

  const uint32_t waves_total = gridDim.x * kWavesPerBlock;
  const uint32_t wave_id = blockIdx.x * kWavesPerBlock + wv;
  const uint32_t ngroups = (trial_count + BATCH - 1u) / BATCH;
  uint32_t g = wave_id, len2 = 0u, len3 = 0u, lql = 0u;          // wave-uniform
  uint32_t h0[3] = {0u, 0u, 0u}, h1[3] = {0u, 0u, 0u};             // decided 0 / 1 in round 1..3 (wave totals)

  for (;;) {
    // ---- pick the work: the deepest full list, fresh round-1 trials, then the partial lists
    uint32_t r, n;
    const uint32_t *src = nullptr;
    if (R >= 3u && len3 >= BATCH) { r = 3u; n = BATCH; src = list3 + (len3 - n); len3 -= n; }
    else if (R >= 2u && len2 >= BATCH) { r = 2u; n = BATCH; src = list2 + (len2 - n); len2 -= n; }
    else if (g < ngroups) { r = 1u; n = trial_count - g * BATCH; n = n < BATCH ? n : BATCH; }
    else if (len2) { r = 2u; n = len2; src = list2; len2 = 0u; }
    else if (len3) { r = 3u; n = len3; src = list3; len3 = 0u; }
    else break;
    r = (uint32_t)__builtin_amdgcn_readfirstlane((int)r);
    n = (uint32_t)__builtin_amdgcn_readfirstlane((int)n);

    // ---- this lane's S trials and their x words (round 1: /start, node.ts:167-188;
    // round r > 1: the coins of round r - 1 after a tie, node.ts:110-111)
    uint32_t toff[S];
    uint32_t w = 0u;
    const uint2 kk = lds_keys(keys);
    const uint64_t tb = lds_u64(keys + 2);
#pragma unroll
    for (uint32_t s = 0; s < S; ++s) {
      const uint32_t e = s * 64u + lane;
      const bool valid = e < n;
      toff[s] = valid ? (src ? src[e] : g * BATCH + e) : 0xFFFFFFFFu;
      uint32_t x = 0u;
      if (valid) {
        const uint64_t tr = tb + toff[s];
        if (r == 1u) {
          x = random_init ? philox4x32_10(kk.x, kk.y, make_uint4((uint32_t)tr, (uint32_t)(tr >> 32), 0u, kStreamInit << 24)).x
                          : fixed1;
        } else {
          x = coin_word(coin_block(kk.x, kk.y, (uint32_t)tr, (uint32_t)(tr >> 32), 0u, r - 1u), r - 1u);
        }
      }
      w |= (x & LIVE) << (s * MM);
    }
    if (r == 1u) g += waves_total;
    // B: +1.0 (0x2) where x = 1, -1.0 (0xA) where x = 0, 0 on unused positions
    const mf_v4i Ez = small_expand(used_mask & ~w);
    const mf_v4i Ex = small_expand(w);
    mf_v4i bx;
#pragma unroll
    for (int v = 0; v < 4; ++v) bx[v] = Ex[v] | Ez[v] | (Ez[v] << 2);

    // ---- R-phase: 8 (c1 - c0) per receiver row -> proposal nibbles (+6 / -6 / 0)
    mf_v4i bp;
    {
      const mf_v16f r0 = mfma_count<3>(A0, bx, zero);
      const mf_v16f r1 = mfma_count<3>(A1, bx, zero);
      bp = mf_v4i{(int)small_pack(r0, 0), (int)small_pack(r0, 8), (int)small_pack(r1, 0), (int)small_pack(r1, 8)};
    }
    mf_v4i babs, bneg, bnabs;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      babs[v] = bp[v] & 0x77777777;                   // |proposal|: 6 unless "?"
      bneg[v] = bp[v] ^ (int)0x88888888u;             // -proposal
      bnabs[v] = bp[v] | (int)0x88888888u;            // -|proposal|
    }
    // ---- P-phase per tile: U (all 1), V (all 0), W (all "?") sign nibbles
    uint32_t un[4], vn[4], wn[4];
#pragma unroll
    for (int T = 0; T < 2; ++T) {
      const mf_v4i A = T == 0 ? A0 : A1;
      const mf_v16f tp = mfma_count(A, babs, cbig);   // 6 (n0 + n1) - (12m - 6)
      const mf_v16f u = mfma_count(A, bp, tp);        // 12 n1 - 12m + 6
      const mf_v16f vv = mfma_count(A, bneg, tp);     // 12 n0 - 12m + 6
      const mf_v16f ww = mfma_count(A, bnabs, four);  // 4 - 6 (n0 + n1)
      un[2 * T] = small_pack(u, 0);
      un[2 * T + 1] = small_pack(u, 8);
      vn[2 * T] = small_pack(vv, 0);
      vn[2 * T + 1] = small_pack(vv, 8);
      wn[2 * T] = small_pack(ww, 0);
      wn[2 * T + 1] = small_pack(ww, 8);
      __builtin_amdgcn_sched_barrier(0);
    }
    // position bits: set where NOT all 1 / NOT all 0 / NOT all "?"
    const uint32_t wu = small_compress(un[0], un[1], un[2], un[3]);
    const uint32_t wvv = small_compress(vn[0], vn[1], vn[2], vn[3]);
    const uint32_t ww = small_compress(wn[0], wn[1], wn[2], wn[3]);

    // ---- per slot: decided (bins 3r + v), tied (next round's list), else the lane path
    const bool last = r >= R;
    uint32_t *next = r == 1u ? list2 : list3;
    uint32_t c1 = 0u, c0 = 0u;
#pragma unroll
    for (uint32_t s = 0; s < S; ++s) {
      const uint32_t fm = LIVE << (s * MM);
      const bool valid = toff[s] != 0xFFFFFFFFu;
      const bool all1 = (wu & fm) == 0u, all0 = (wvv & fm) == 0u, tie = (ww & fm) == 0u;
      c1 += (valid && all1) ? 1u : 0u;
      c0 += (valid && all0) ? 1u : 0u;
      const bool to_next = valid && tie && !last && !all1 && !all0;
      const bool to_lane = valid && !all1 && !all0 && !to_next;
      const uint64_t bn = ballot(to_next), bl = ballot(to_lane);
      if (to_next) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bn >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bn, 0u));
        next[(r == 1u ? len2 : len3) + rank] = toff[s];
      }
      if (to_lane) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0u));
        lq[lql + rank] = toff[s];
      }
      if (r == 1u) len2 += (uint32_t)__builtin_popcountll(bn);
      else len3 += (uint32_t)__builtin_popcountll(bn);
      lql += (uint32_t)__builtin_popcountll(bl);
    }
    // wave totals of the decided counts: bit-sliced ballots (c <= S <= 8)
    uint32_t t1 = 0u, t0 = 0u;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      t1 += (uint32_t)__builtin_popcountll(ballot((c1 >> b) & 1u)) << b;
      t0 += (uint32_t)__builtin_popcountll(ballot((c0 >> b) & 1u)) << b;
    }
    if (r == 1u) { h1[0] += t1; h0[0] += t0; }
    else if (r == 2u) { h1[1] += t1; h0[1] += t0; }
    else { h1[2] += t1; h0[2] += t0; }

    // ---- lane path, 64 queued trials at a time (every lane busy)
    while (lql >= 64u) {
      lql -= 64u;
      const uint32_t t = lq[lql + lane];
      const uint64_t tr = lds_u64(keys + 2) + t;
      const uint2 k2 = lds_keys(keys);
      uint32_t x = fixed1;
      if (random_init) x = philox4x32_10(k2.x, k2.y, make_uint4((uint32_t)tr, (uint32_t)(tr >> 32), 0u, kStreamInit << 24)).x & LIVE;
      const uint32_t bin = small_lane_trial<MM>(k2.x, k2.y, tr, x, F, k_max);
      atomicAdd(&lhist[bin & 0x7FFFFFFFu], 1u);
      if (bin >> 31) atomicAdd(&lhist[hist_len - 1u], 1u);
    }
  }
  // ---- the rest of the lane-path queue
  if (lane < lql) {
    const uint32_t t = lq[lane];
    const uint64_t tr = lds_u64(keys + 2) + t;
    const uint2 k2 = lds_keys(keys);
    uint32_t x = fixed1;
    if (random_init) x = philox4x32_10(k2.x, k2.y, make_uint4((uint32_t)tr, (uint32_t)(tr >> 32), 0u, kStreamInit << 24)).x & LIVE;
    const uint32_t bin = small_lane_trial<MM>(k2.x, k2.y, tr, x, F, k_max);
    atomicAdd(&lhist[bin & 0x7FFFFFFFu], 1u);
    if (bin >> 31) atomicAdd(&lhist[hist_len - 1u], 1u);
  }
  // outcome bins 3r + v of the matrix-core rounds (lane l < 9 adds one of them)
  {
    const uint32_t rr = lane / 2u + 1u;
    uint32_t c = 0u;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (lane == 2u * q) c = h0[q];
      if (lane == 2u * q + 1u) c = h1[q];
    }
    if (lane < 6u && c) atomicAdd(&lhist[3u * rr + (lane & 1u)], c);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < hist_len; i += blockDim.x) {
    const uint32_t c = lhist[i];
    if (c) atomicAdd(&p.hist[i], (unsigned long long)c);
  }
}

template <int MM>
hipError_t launch_mfma_small_m(const KParams &p, int grid, hipStream_t s) {
  hipLaunchKernelGGL((benor_mfma_small_kernel<MM>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  return hipGetLastError();
}

}  // namespace benor
