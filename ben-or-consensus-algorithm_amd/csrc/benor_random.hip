// benor_random.hip -- random-delivery kernel for the Bernoulli + fix-up sampler
// (r04).
//
// Same definition, bit for bit, as oracle/benor_oracle.c oracle_delivery_mask
// sampler (b) and the r02 kernel (benor_kernels.hip benor_random_kernel, which
// keeps the Floyd sampler): every live receiver tallies, per phase, a uniform
// q-subset of the m live senders -- a Bernoulli(a/16) mask from Philox stream 2
// followed by exact fix-up flips at uniform sender indices.  Reference
// semantics: node.ts:52-69 (R-phase tally), :88-113 (P-phase), with "the first
// N-F arrivals" of SURVEY §8f #4.
//
// One wave = one trial, lane l of receiver group j = live node 64 j + l.  What
// changed against r02 (the same bits, fewer instructions):
//
//   * Philox: the delivery counter is {trial_lo, trial_hi, blk | round << 16 |
//     phase << 31, node | 2 << 24} (r04 layout: the receiver in the last word,
//     the block in the third), so the first rounds' products that do not
//     involve the receiver are wave-uniform (scalar unit) and the one that
//     does not involve the block is computed once per receiver-phase
//     (dlv_block): 15 v_mad_u64_u32 and 17 xors per block instead of 20 and 20.
//   * fix-up: one ds_mskor_rtn_b32 per field tests and flips in one LDS op
//     (mask = the sender's bit, data = its target value), so a sender named
//     twice is refused by the LDS state itself, in stream order.  The fields
//     of a Philox block are issued speculatively without waiting for the
//     quota; a lane that passes its quota inside the block undoes its last
//     accepted flips (they are distinct senders), which leaves exactly the
//     sequential definition's result.
//   * out-of-range indices (idx >= m when m is not a power of two) need no
//     compare: the bitset has 2^b / 32 rows and every bit >= m holds the
//     lane's refusal value (1 when it removes, 0 when it adds), so such a
//     field is refused by the same test.  Padding bits never reach a tally:
//     the sender planes have no bit >= m.
//   * tally: c1 from one plane when no vote can be "?" (every R-phase after
//     round 1, and round 1 without "?" inputs): c0 = q - c1.
#include "benor_device.h"

namespace benor {

namespace {

constexpr uint32_t kM0 = 0xD2511F53u, kM1 = 0xCD9E8D57u, kW0 = 0x9E3779B9u, kW1 = 0xBB67AE85u;

typedef __attribute__((address_space(3))) uint32_t lds_word;

// The delivery stream's counter is {tlo, thi, c2 = block | round << 16 |
// phase << 31, c3 = node | 2 << 24} (oracle_delivery_mask): within a trial's
// (round, phase) only c3 differs between receivers and only c2 between
// blocks.  So, per Philox4x32-10 block:
//   round 1: M0 tlo is per trial; M1 c2 is per block (wave-uniform);
//            x1 = hi(M1 c2) ^ thi ^ K0[1] is wave-uniform; z1 = hi(M0 tlo) ^ c3 ^ K1[1]
//            is per receiver but the same for every block;
//   round 2: M0 x1 is per block (uniform); M1 z1 is per receiver (once per
//            receiver-phase); x2 = hi(M1 z1) ^ lo(M1 c2) ^ K0[2] -- one xor;
//   round 3: M1 z2 is per block (uniform); M0 x2 is the first per-lane product;
//   rounds 4..10 as Philox.
// 15 v_mad_u64_u32 and 17 xors per block instead of 20 and 20; the uniform
// products go to the scalar unit.
struct DlvUni {            // per (trial, round, phase), wave-uniform
  uint32_t k0, k1, thi, c2, a1, w1;   // a1 = hi(M0 tlo) ^ K1[1], w1 = lo(M0 tlo)
};
struct DlvRecv {           // per receiver-phase (lane)
  uint32_t h1, l1;         // M1 z1, z1 = c3 ^ a1
};

__device__ __forceinline__ uint32_t sgpr(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

__device__ __forceinline__ DlvUni dlv_uniforms(uint32_t k0, uint32_t k1, uint32_t tlo, uint32_t thi, uint32_t r,
                                              uint32_t phase) {
  const uint64_t p0 = (uint64_t)kM0 * tlo;
  DlvUni u;
  u.k0 = sgpr(k0);
  u.k1 = sgpr(k1);
  u.thi = sgpr(thi);
  u.c2 = sgpr(((r & 0x7FFFu) << 16) | ((phase & 1u) << 31));
  u.a1 = sgpr((uint32_t)(p0 >> 32) ^ k1);
  u.w1 = sgpr((uint32_t)p0);
  return u;
}

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t m) { return (uint64_t)a * m; }

__device__ __forceinline__ DlvRecv dlv_receiver(const DlvUni &u, uint32_t node) {
  const uint32_t z1 = (node & 0xFFFu) ^ (kStreamDelivery << 24) ^ u.a1;
  const uint64_t p = mad64(z1, kM1);
  return DlvRecv{(uint32_t)(p >> 32), (uint32_t)p};
}

__device__ __forceinline__ uint32_t xor_s(uint32_t v, uint32_t s) {   // v ^ s, s wave-uniform
  uint32_t r;
  asm("v_xor_b32 %0, %1, %2" : "=v"(r) : "s"(s), "v"(v));
  return r;
}

// Philox4x32-10 block `blk` of the receiver's delivery stream -- the value of
// philox4x32_10(k0, k1, {tlo, thi, c2 | blk, c3}).
__device__ __forceinline__ uint4 dlv_block(const DlvUni &u, const DlvRecv &v, uint32_t blk) {
  const uint32_t k0 = u.k0, k1 = u.k1;
  // wave-uniform part (scalar unit)
  const uint64_t P = (uint64_t)kM1 * sgpr(u.c2 | blk);            // round 1: M1 c2
  const uint32_t x1 = (uint32_t)(P >> 32) ^ u.thi ^ k0;
  const uint64_t Q = (uint64_t)kM0 * x1;                           // round 2: M0 x1
  const uint32_t z2 = (uint32_t)(Q >> 32) ^ u.w1 ^ (k1 + kW1);
  const uint64_t S = (uint64_t)kM1 * z2;                           // round 3: M1 z2
  const uint32_t s_x2 = sgpr((uint32_t)P ^ (k0 + kW0));
  const uint32_t s_x3 = sgpr((uint32_t)(S >> 32) ^ (k0 + 2u * kW0));
  const uint32_t s_z3 = sgpr((uint32_t)Q ^ (k1 + 2u * kW1));
  const uint32_t s_x4 = sgpr((uint32_t)S ^ (k0 + 3u * kW0));
  // round 2: x2 = hi(M1 z1) ^ lo(M1 c2) ^ K0[2]; y2 = lo(M1 z1)
  const uint32_t x2 = xor_s(v.h1, s_x2);
  // round 3: x3 = hi(M1 z2) ^ y2 ^ K0[3]; z3 = hi(M0 x2) ^ lo(M0 x1) ^ K1[3]
  const uint64_t a = mad64(x2, kM0);
  const uint32_t x3 = xor_s(v.l1, s_x3), z3 = xor_s((uint32_t)(a >> 32), s_z3), w3 = (uint32_t)a;
  // round 4: y3 = lo(M1 z2) is uniform (in s_x4)
  const uint64_t p0 = mad64(x3, kM0), p1 = mad64(z3, kM1);
  uint4 c = make_uint4(xor_s((uint32_t)(p1 >> 32), s_x4), (uint32_t)p1,
                       xor3_key((uint32_t)(p0 >> 32), w3, k1 + 3u * kW1), (uint32_t)p0);
#pragma unroll
  for (uint32_t r = 4; r < 10; ++r) {
    const uint64_t q0 = mad64(c.x, kM0), q1 = mad64(c.z, kM1);
    c = make_uint4(xor3_key((uint32_t)(q1 >> 32), c.y, k0 + r * kW0), (uint32_t)q1,
                   xor3_key((uint32_t)(q0 >> 32), c.w, k1 + r * kW1), (uint32_t)q0);
  }
  return c;
}

__device__ __forceinline__ uint32_t word_of(const uint4 &b, int j) {
  return j == 0 ? b.x : j == 1 ? b.y : j == 2 ? b.z : b.w;
}

// r = a_i ? (~u | r) : (~u & r), a_i wave-uniform (amask = 0 or ~0): one
// v_bitop3_b32 (LUT over (u, r, amask)).
__device__ __forceinline__ uint32_t cmp_step(uint32_t u, uint32_t r, uint32_t amask) {
  // LUT index u << 2 | r << 1 | a (S0 << 2 | S1 << 1 | S2):
  //   0:0  1:1  2:1  3:1  4:0  5:0  6:0  7:1  ->  0b10001110 = 0x8E
  uint32_t o;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x8E" : "=v"(o) : "v"(u), "v"(r), "s"(amask));
  return o;
}

// The first step folded with r = ~u0: a ? !(u1 & u0) : !(u1 | u0).  LUT index
// u1 << 2 | u0 << 1 | a (v_bitop3 indexes S0 << 2 | S1 << 1 | S2):
//   0:1  1:1  2:0  3:1  4:0  5:1  6:0  7:0  ->  0b00101011 = 0x2B
__device__ __forceinline__ uint32_t cmp_step_first(uint32_t u1, uint32_t u0, uint32_t amask) {
  uint32_t o;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x2B" : "=v"(o) : "v"(u1), "v"(u0), "s"(amask));
  return o;
}

// This lane's bitset row of field bits [off, off + w): lb + (field << 8), one
// v_bfe_u32 and one v_lshl_add_u32 (the compiler's shift / and / add is three).
__device__ __forceinline__ uint32_t row_addr(uint32_t wd, uint32_t off, uint32_t w, uint32_t lb) {
  const uint32_t t = __builtin_amdgcn_ubfe(wd, off, w);
  uint32_t a;
  asm("v_lshl_add_u32 %0, %1, 8, %2" : "=v"(a) : "v"(t), "v"(lb));
  return a;
}

// 1 << (s & 31) as the all-VGPR VOP2 v_lshlrev_b32 (the shift reads s's low 5 bits).
__device__ __forceinline__ uint32_t bit_of(uint32_t s, uint32_t one) {
  uint32_t r;
  asm("v_lshlrev_b32 %0, %1, %2" : "=v"(r) : "v"(s), "v"(one));
  return r;
}

__device__ __forceinline__ uint32_t mskor_rtn(uint32_t addr, uint32_t mask, uint32_t data) {
  uint32_t old;
  asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3" : "=v"(old) : "v"(addr), "v"(mask), "v"(data) : "memory");
  return old;
}

// One receiver's delivered-sender mask (oracle_delivery_mask, sampler (b)),
// left in this lane's column of the bitset B ([row][lane], 256 bytes a row),
// then its tally of the planes (X records {x0lo, x0hi, x1lo, x1hi} per 64
// senders).  NW = 4 - tz(a) stream words per mask word; B = ceil(log2 m)
// bits per fix-up field, PER = floor(32 / B) fields per stream word.
template <int NW, int B>
__device__ __forceinline__ void bern_tally(const uint4 *__restrict__ plane, uint32_t lb, uint32_t m, uint32_t q,
                                           uint32_t W32, uint32_t rows, uint32_t amask1, uint32_t amask2,
                                           uint32_t amask3, bool active, bool one_plane, const DlvUni &u,
                                           uint32_t node, uint32_t &c0, uint32_t &c1) {
  constexpr int L = NW == 3 ? 12 : 4, NB = L / 4, MW = L / NW;   // stream words, blocks, mask words per super-block
  constexpr int PER = 32 / B, NF = 4 * PER;
  const DlvRecv rv = dlv_receiver(u, node);
  const uint32_t tail = m & 31u ? (1u << (m & 31u)) - 1u : ~0u;   // the last mask word's live bits
  // ---- Bernoulli(a/16) mask: bit = (u < a), bits tz(a).. 3 of u from the
  // mask word's NW stream words, lowest first (oracle: r = ~u_tz; then
  // r = a_i ? (~u | r) : (~u & r)).
  uint32_t c = 0, blk = 0;
  for (uint32_t w0 = 0; w0 < W32; w0 += MW, blk += NB) {
    uint32_t s[L];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (j == 0 || w0 + (uint32_t)((4 * j) / NW) < W32) {    // blocks a partial super-block needs
        const uint4 bb = dlv_block(u, rv, blk + (uint32_t)j);
        s[4 * j] = bb.x, s[4 * j + 1] = bb.y, s[4 * j + 2] = bb.z, s[4 * j + 3] = bb.w;
      }
    }
#pragma unroll
    for (int t = 0; t < MW; ++t) {
      const uint32_t w = w0 + (uint32_t)t;
      if (w < W32) {
        uint32_t r;
        if constexpr (NW >= 2) r = cmp_step_first(s[t * NW + 1], s[t * NW], NW == 4 ? amask1 : NW == 3 ? amask2 : amask3);
        else r = ~s[t * NW];
        if constexpr (NW >= 3) r = cmp_step(s[t * NW + 2], r, NW == 4 ? amask2 : amask3);
        if constexpr (NW >= 4) r = cmp_step(s[t * NW + 3], r, amask3);
        if (w + 1u == W32) r &= tail;
        *(lds_word *)(uintptr_t)(lb + w * 256u) = r;
        c = tally(r, c);
      }
    }
  }
  blk = (W32 * (uint32_t)NW + 3u) >> 2;          // the first block after the mask's last stream word
  // ---- exact fix-up (c != q): fields from the Philox block after the mask's
  // last word; each names a sender idx, accepted when its bit is the
  // refusal's opposite (remove a member while c > q, add a non-member while
  // c < q), until |c - q| flips were accepted.
  const bool rm = c > q;
  uint32_t rem = active ? (rm ? c - q : q - c) : 0u;
  const uint32_t fill = rm ? 0u : ~0u;          // padding (bits >= m) refuses every field
  {
    const uint32_t n = m & 31u;
    if (n) {                                     // the last word's bits >= m
      lds_word *pw = (lds_word *)(uintptr_t)(lb + (W32 - 1u) * 256u);
      *pw = *pw | (fill & ~((1u << n) - 1u));
    }
    for (uint32_t w = W32; w < rows; ++w) *(lds_word *)(uintptr_t)(lb + w * 256u) = fill;
  }
  uint32_t addm = rm ? 0u : ~0u;                 // data = bit when adding
  uint32_t one = 1u;                              // a VGPR 1: 1 << s as an all-VGPR v_lshlrev_b32
  asm volatile("" : "+v"(one), "+v"(addm));       // VGPRs: v_and_b32 (VOP2) for data, not v_cndmask
  for (; __any(rem != 0u); ++blk) {
    const uint4 bb = dlv_block(u, rv, blk);
    if (rem != 0u) {
      uint32_t addr[NF], bit[NF], data[NF], old[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        // field f: bits [off, off + B) of stream word f / PER; sender idx = row
        // idx >> 5 (the field's top B - 5 bits), bit idx & 31 (its low 5 bits)
        const uint32_t wd = word_of(bb, f / PER);
        const uint32_t off = (uint32_t)(f % PER) * B;   // a constant once unrolled
        addr[f] = row_addr(wd, off + 5u, B - 5u, lb);
        bit[f] = off ? bit_of(__builtin_amdgcn_ubfe(wd, off, 5u), one) : bit_of(wd, one);
        data[f] = bit[f] & addm;
        old[f] = mskor_rtn(addr[f], bit[f], data[f]);
      }
      // one wait for the NF returns (their consumers read the values after it)
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(old[0]), "+v"(old[1]), "+v"(old[2]), "+v"(old[3]), "+v"(old[4]), "+v"(old[5]),
                     "+v"(old[6]), "+v"(old[7]) :: "memory");
      if constexpr (NF > 8)
        asm volatile("" : "+v"(old[8 % NF]), "+v"(old[9 % NF]), "+v"(old[10 % NF]), "+v"(old[11 % NF]) :: "memory");
      if constexpr (NF > 12)
        asm volatile("" : "+v"(old[12 % NF]), "+v"(old[13 % NF]), "+v"(old[14 % NF]), "+v"(old[15 % NF]) :: "memory");
      uint32_t cnt = 0, acc[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        acc[f] = (old[f] ^ data[f]) & bit[f];            // the flip happened
        cnt = tally(acc[f], cnt);
      }
      if (cnt > rem) {                           // past the quota in this block: undo the last accepted
        uint32_t excess = cnt - rem;
#pragma unroll
        for (int f = NF - 1; f >= 0; --f) {
          if (excess != 0u && acc[f] != 0u) {
            __hip_atomic_fetch_xor((lds_word *)(uintptr_t)addr[f], bit[f], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WAVEFRONT);
            --excess;
          }
        }
        rem = 0u;
      } else {
        rem -= cnt;
      }
    }
  }
  // ---- tally (node.ts:52-69 / :88-113): the delivered senders' votes
  uint32_t a0 = 0, a1 = 0;
  for (uint32_t w = 0; w < W32; w += 2u) {
    const uint4 rc = plane[w >> 1];
    const uint32_t d0 = *(const lds_word *)(uintptr_t)(lb + w * 256u);
    a1 = tally(d0 & rc.z, a1);
    if (!one_plane) a0 = tally(d0 & rc.x, a0);
    if (w + 1u < W32) {
      const uint32_t d1 = *(const lds_word *)(uintptr_t)(lb + (w + 1u) * 256u);
      a1 = tally(d1 & rc.w, a1);
      if (!one_plane) a0 = tally(d1 & rc.y, a0);
    }
  }
  c0 = one_plane ? q - a1 : a0;
  c1 = a1;
}

template <int NW, int B>
__global__ void __launch_bounds__(256) benor_random_bern_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t m = p.m, F = p.F, W = p.W, q = p.q;
  const uint32_t W32 = (m + 31u) >> 5, rows = p.rd_rows;

  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  uint4 *X = reinterpret_cast<uint4 *>(smem + p.hist_bytes + wv * p.wave_bytes);   // [W]
  uint4 *P = X + W;                                                                 // [W]
  uint32_t *bits = reinterpret_cast<uint32_t *>(P + W);                             // [rows][64] bitset
  const uint32_t lb = (uint32_t)(uintptr_t)(lds_word *)bits + lane * 4u;

  for (uint32_t i = threadIdx.x; i < p.hist_len; i += blockDim.x) lhist[i] = 0u;
  __syncthreads();

  uint64_t expect = 0ull;                          // groups holding a live receiver for this lane
  for (uint32_t j = 0; j < W; ++j)
    if (j * 64u + lane < m) expect |= 1ull << j;
  // a's bits above tz(a), as wave-uniform masks (cmp_step)
  const uint32_t a = p.rd_a, tz = 4u - (uint32_t)NW;
  const uint32_t am1 = ((a >> (tz + 1u)) & 1u) ? ~0u : 0u;   // used when NW = 4 (bit 1)
  const uint32_t am2 = ((a >> (4u - 2u)) & 1u) ? ~0u : 0u;   // bit 2 (NW >= 3)
  const uint32_t am3 = ((a >> 3u) & 1u) ? ~0u : 0u;          // bit 3 (NW >= 2)

  const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
  const uint64_t waves_total = (uint64_t)gridDim.x * kWavesPerBlock;
  const bool r1_plain = p.init_mode == BO_INIT_RANDOM || p.init_q == 0u;   // round 1 x has no "?"

  for (uint64_t t = (uint64_t)blockIdx.x * kWavesPerBlock + wv; t < p.trial_count; t += waves_total) {
    const uint64_t trial = p.trial_begin + t;
    const uint32_t tlo = sgpr((uint32_t)trial), thi = sgpr((uint32_t)(trial >> 32));
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
      {
        const DlvUni u = dlv_uniforms(k0, k1, tlo, thi, r, 0u);
        const bool one = r > 1u || r1_plain;
        for (uint32_t j = 0; j < W; ++j) {
          const uint32_t c = j * 64u + lane;
          const bool active = c < m;
          const uint32_t node = active ? p.live_ids[c] : 0u;
          uint32_t a0, a1;
          bern_tally<NW, B>(X, lb, m, q, W32, rows, am1, am2, am3, active, one, u, node, a0, a1);
          const uint64_t vm = group_mask(j, m);
          const uint64_t p0 = ballot(a0 > a1) & vm;
          const uint64_t p1 = ballot(a1 > a0) & vm;
          if (lane == 0) P[j] = rec(p0, p1);
        }
      }
      // ---- P-phase ("voting phase", node.ts:83-158)
      {
        const DlvUni u = dlv_uniforms(k0, k1, tlo, thi, r, 1u);
        for (uint32_t j = 0; j < W; ++j) {
          const uint32_t c = j * 64u + lane;
          const bool active = c < m;
          const uint32_t node = active ? p.live_ids[c] : 0u;
          uint32_t a0, a1;
          bern_tally<NW, B>(P, lb, m, q, W32, rows, am1, am2, am3, active, false, u, node, a0, a1);
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

template <int NW, int B>
hipError_t launch_nw_b(const KParams &p, int grid, hipStream_t s) {
  const void *fn = reinterpret_cast<const void *>(&benor_random_bern_kernel<NW, B>);
  if (p.lds_bytes > 64u * 1024u) {
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds_bytes);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((benor_random_bern_kernel<NW, B>), dim3(grid), dim3(64 * kWavesPerBlock), p.lds_bytes, s, p);
  return hipGetLastError();
}

template <int NW>
hipError_t launch_nw(const KParams &p, int grid, hipStream_t s) {
  switch (p.rd_b) {   // m in [128, 4096]: b = ceil(log2 m) in 7..12 (b = 7 only at m = 128, q = 64)
    case 7: return launch_nw_b<NW, 7>(p, grid, s);
    case 8: return launch_nw_b<NW, 8>(p, grid, s);
    case 9: return launch_nw_b<NW, 9>(p, grid, s);
    case 10: return launch_nw_b<NW, 10>(p, grid, s);
    case 11: return launch_nw_b<NW, 11>(p, grid, s);
    default: return launch_nw_b<NW, 12>(p, grid, s);
  }
}

}  // namespace

uint32_t random_bern_rows(uint32_t m, uint32_t b) {
  const uint32_t W32 = (m + 31u) >> 5, r = (1u << b) >> 5;
  return r > W32 ? r : W32;
}

hipError_t launch_random_bern(const KParams &p, int grid, hipStream_t s) {
  if (p.rd_a == 0u || p.rd_b < 7u || p.rd_b > 12u || p.rd_rows < random_bern_rows(p.m, p.rd_b))
    return hipErrorInvalidValue;
  const uint32_t tz = (uint32_t)__builtin_ctz(p.rd_a);
  switch (4u - tz) {
    case 4: return launch_nw<4>(p, grid, s);
    case 3: return launch_nw<3>(p, grid, s);
    case 2: return launch_nw<2>(p, grid, s);
    default: return launch_nw<1>(p, grid, s);
  }
}

}  // namespace benor
