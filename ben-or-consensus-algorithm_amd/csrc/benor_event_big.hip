// benor_event_big.hip -- event-level mode for 256 < N <= 4096, and live runs at any N
// (r04).
//
// The reference's GET /stop (node.ts:191-194) lands on a running consensus at
// any network size; from then on the node drops every message (node.ts:45).
// This kernel runs the message-granular model of oracle/benor_oracle.c (iii)
// event_trial() -- the literal POST /message handler (node.ts:45-158), one
// delivery per event in the seeded order, scheduled stops applied at their
// delivery counts -- for networks too large for benor_event_kernel (one lane
// per trial, N <= 256).  Definition and its bit-exact checks: the oracle.
//
// One wave = one trial (a 64-thread workgroup):
//   * the message pool (uniform pick, swap-remove) lives in the workgroup's
//     HBM scratch slice: 4N^2 + 64 u32 messages, to | ph << 12 | x << 13 |
//     (k & 3) << 15 (k is recovered from the completion round `cur`, as in
//     benor_event_kernel: a message to a running node is for [cur, cur + 2]).
//     A pool of at most kEventBigLdsPool bytes (N <= 78: the reference's own
//     network sizes, live runs) lives in LDS instead (LP), so a batch's pool
//     loads are LDS reads rather than L2 round trips;
//   * per-node state lives in LDS: inbox counters {c0, c1, len} per phase
//     (13 bits each, bit 63 = killed), x, k, the compact index for coins, and
//     node bitsets (killed, decided, completion of rounds cur .. cur + 3).
//     Every initially live node's message is needed for a quorum (exactly F
//     faulty, launchNodes.ts:12-13), so a node's inbox for a phase holds one
//     round at a time: R_k and R_{k+1} (P_k and P_{k+1}) are never in flight
//     to it together, and the slot is cleared when its trigger fires;
//   * the event chain is sequential (each pick depends on the pool's length,
//     which a trigger changes).  Events go in batches of up to 64: lane i
//     computes the pick of event e + i assuming no trigger (splitmix64 is a
//     counter: state e + i is state e + (i + 1) * gamma) and loads both pool
//     words the swap-remove touches, so one HBM round trip serves 64 events
//     (and the next batch's words are loaded while this one resolves).  The
//     batch's messages are resolved in parallel -- which earlier event of the
//     batch last wrote a lane's pick or tail position, by a scan that an LDS
//     bitmap of the picks skips in most batches, and pointer jumping along the
//     swap-remove chains -- and its deliveries are applied at once unless an
//     inbox reaches its quorum inside the batch (then the batch replays one
//     delivery at a time up to that trigger).  A trigger ends the batch: the
//     used events' writes go back, the triggered broadcast is appended, and
//     the next batch starts after it.  Batches also end before a scheduled stop.
//   * r04-r05 live runs also ran here (a host-mapped mailbox polled between
//     batches); since r06 they run on csrc/benor_event_live.hip, and this
//     kernel serves batch event plans (many trials) only.
#include "benor_device.h"

namespace benor {

namespace {

constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ull;
constexpr uint64_t kC13 = (1ull << 13) - 1ull;
constexpr uint64_t kKilled = 1ull << 63;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t lane) {   // v of `lane`, wave-uniform
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }   // v_min_u32
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }   // v_max_u32

// All-ones when x == 0 (else 0), and all-ones when (int)(a - b) < 0 (|a - b| <
// 2^31) -- VALU arithmetic in asm, so the compiler cannot turn them back into
// compares feeding v_cndmask_b32 (a VCC / SGPR-pair select, ~24 cycles per wave
// instruction on gfx950 against 2-4 here).
__device__ __forceinline__ uint32_t zero_mask(uint32_t x) {
  uint32_t r;
  asm("v_min_u32 %0, 1, %1\n\tv_add_u32 %0, -1, %0" : "=&v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ uint32_t below_mask(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_sub_u32 %0, %1, %2\n\tv_ashrrev_i32 %0, 31, %0" : "=&v"(r) : "v"(a), "v"(b));
  return r;
}

// The wave's LDS ordering point (one wave per workgroup: a fence and a wave
// barrier).
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

struct BigState {
  uint64_t *ibox;     // [N][2] {c0, c1, len} per phase, bit 63 killed
  int8_t *xs;         // [N]
  int16_t *ks;        // [N]
  uint16_t *cidx;     // [N] compact live index (coins)
  uint64_t *killed;   // [64]
  uint64_t *decided;  // [64]
  uint64_t *comp;     // [4][64] completion of round k at k & 3
  uint32_t *picks;    // [2048] a batch's pick positions, low 16 bits as a bitmap
  uint32_t *wrote;    // [2048] the positions a batch wrote back, likewise
  uint64_t *rstops;   // [ev_rstops] a random /stop schedule (event << 12 | node), ~0 once applied
  uint64_t *rset;     // [64] its Floyd set over compact live indices
};

}  // namespace

template <bool LP>
__global__ void __launch_bounds__(64) benor_event_big_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t *lhist = reinterpret_cast<uint32_t *>(smem);
  const uint32_t N = p.N, F = p.F, quorum = p.N - p.F, m = p.m;
  const uint32_t NWd = (N + 63u) >> 6;                       // bitset words (<= 64: one per lane)
  for (uint32_t i = lane; i < p.hist_len; i += 64u) lhist[i] = 0u;
  __syncthreads();   // the only workgroup barrier: below, the wave syncs with itself (wsync)

  BigState S;
  unsigned char *q = smem + p.hist_bytes;
  S.ibox = reinterpret_cast<uint64_t *>(q);
  S.killed = S.ibox + 2u * N;
  S.decided = S.killed + 64;
  S.comp = S.decided + 64;
  S.ks = reinterpret_cast<int16_t *>(S.comp + 4 * 64);
  S.cidx = reinterpret_cast<uint16_t *>(S.ks + ((N + 3u) & ~3u));
  S.xs = reinterpret_cast<int8_t *>(S.cidx + ((N + 3u) & ~3u));
  S.picks = reinterpret_cast<uint32_t *>(S.xs + ((N + 15u) & ~15u));
  S.wrote = S.picks + 2048;
  S.rset = reinterpret_cast<uint64_t *>(S.wrote + 2048);
  S.rstops = S.rset + 64;
  for (uint32_t i = lane; i < 2048u; i += 64u) S.picks[i] = 0u;
  const uint64_t allw = lane < NWd ? (N >= 64u * (lane + 1u) ? ~0ull : (1ull << (N - 64u * lane)) - 1ull) : 0ull;
  const uint64_t wmask = NWd >= 64u ? ~0ull : ((1ull << NWd) - 1ull);   // lanes holding a bitset word
  const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
  uint32_t *pool;
  if constexpr (LP) pool = reinterpret_cast<uint32_t *>(S.rstops + p.ev_rstops);   // after the LDS state
  else pool = p.scratch + (uint64_t)blockIdx.x * p.ev_stride;
  const uint32_t cap = p.ev_cap;

  // a | b == all, over the bitset words (one per lane)
  auto full = [&](const uint64_t *a, const uint64_t *b) {
    const bool ok = lane >= NWd || ((a[lane] | b[lane]) == allw);
    return (__ballot(ok) & wmask) == wmask;
  };

  for (uint64_t t = blockIdx.x; t < p.trial_count; t += gridDim.x) {
    const uint64_t trial = p.trial_begin + t;
    const uint32_t tlo = (uint32_t)trial, thi = (uint32_t)(trial >> 32);
    // ---- node.ts:21-26: faulty nodes killed, live nodes x = initial value
    for (uint32_t w = lane; w < 64u; w += 64u) {
      S.killed[w] = w < NWd ? allw : 0ull;   // every node, then the live ones cleared
      S.decided[w] = 0ull;
      for (int r = 0; r < 4; ++r) S.comp[r * 64 + w] = 0ull;
    }
    for (uint32_t i = lane; i < N; i += 64u) {
      S.xs[i] = -1;
      S.ks[i] = -1;
      S.ibox[2u * i] = kKilled;
      S.ibox[2u * i + 1u] = kKilled;
    }
    wsync();
    for (uint32_t c = lane; c < m; c += 64u) {
      const uint32_t i = p.live_ids[c];
      int8_t v;
      if (p.init_mode == BO_INIT_RANDOM) {      // oracle_random_init: m <= 32 a block per four trials,
        if (m <= 32u) {                         // else word c >> 5 of the trial's stream 1
          v = (int8_t)((init_word_small(k0, k1, trial) >> c) & 1u);
        } else {
          const uint4 ir = philox4x32_10<false>(k0, k1, make_uint4(tlo, thi, c >> 7, kStreamInit << 24));
          v = (int8_t)((coin_word_v(ir, ((c >> 5) & 3u) + 1u) >> (c & 31u)) & 1u);
        }
      } else {
        v = p.init_x[i];
      }
      S.xs[i] = v;
      S.ks[i] = 1;                              // /start: k = 1 (node.ts:172)
      S.cidx[i] = (uint16_t)c;
      S.ibox[2u * i] = 0ull;
      S.ibox[2u * i + 1u] = 0ull;
      __hip_atomic_fetch_and(reinterpret_cast<unsigned long long *>(&S.killed[i >> 6]), ~(1ull << (i & 63u)),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    wsync();
    // ---- /start (node.ts:167-188): every live node broadcasts its x, in node order
    uint32_t len = 0;
    for (uint32_t c = 0; c < m; ++c) {
      const uint32_t i = p.live_ids[c];
      const uint32_t body = ((uint32_t)(S.xs[i] & 3) << 13) | (1u << 15);
      for (uint32_t to = lane; to < N; to += 64u) pool[len + to] = to | body;
      len += N;
    }
    uint64_t rng;
    {
      const uint4 o = philox4x32_10<false>(k0, k1, make_uint4(tlo, thi, 0u, kStreamOrder << 24));
      rng = (((uint64_t)o.x << 32) | o.y) ^ 0xD1B54A32D192ED03ull;
    }
    // ---- the /stop schedule: explicit (crash_at, sorted on the host, the same
    // for every trial) or random per trial (crash_count, oracle event_trial):
    // Floyd over compact live indices from Philox stream 4, then one uniform
    // delivery count in [0, crash_window) per pick, in pick order.  next_key is
    // the schedule's smallest unapplied (event << 12 | node), ~0 when none.
    const uint32_t kr = p.ev_rstops;
    if (kr) {
      S.rset[lane] = 0ull;
      wsync();
      if (lane == 0u) {
        DStream ds;
        ds.k0 = k0; ds.k1 = k1; ds.c0 = tlo; ds.c1 = thi; ds.c2 = 0u; ds.c3 = kStreamCrash << 24; ds.widx = 0;
        ds.sh = 12u;
        for (uint32_t j = m - kr, n = 0; j < m; ++j, ++n) {
          const uint32_t tt = ds.uniform(j + 1u);
          const uint32_t idx = ((S.rset[tt >> 6] >> (tt & 63u)) & 1ull) ? j : tt;
          S.rset[idx >> 6] |= 1ull << (idx & 63u);
          S.rstops[n] = idx;
        }
        for (uint32_t n = 0; n < kr; ++n) {
          const uint32_t when = ds.uniform(p.crash_window);
          S.rstops[n] = ((uint64_t)when << 12) | p.live_ids[(uint32_t)S.rstops[n]];
        }
      }
      wsync();
    }
    auto rstops_min = [&]() {                   // wave-uniform minimum of the random schedule
      uint64_t v = ~0ull;
      for (uint32_t i = lane; i < kr; i += 64u) v = v < S.rstops[i] ? v : S.rstops[i];
      for (int off = 32; off >= 1; off >>= 1) {
        const uint64_t o = __shfl_xor(v, off);
        v = v < o ? v : o;
      }
      return v;
    };
    uint32_t next = 0;
    uint64_t next_key = kr ? rstops_min() : (p.ev_nstops ? p.ev_stops[0] : ~0ull);
    __threadfence_block();
    uint32_t cur = 1, R = 0, halted = 0;
    // the next batch's picks and pool words, loaded while this batch resolves
    // (valid when it starts at pf_e with pf_len messages and pf_b events)
    uint32_t pf_pk = 0u, pf_pv = 0u, pf_tv = 0u, pf_len = 0u, wq = 0xFFFFFFFFu;
    uint64_t pf_e = ~0ull, pf_b = 0ull;
    for (uint32_t i = lane; i < 2048u; i += 64u) S.wrote[i] = 0u;
    bool overflow = false;
    uint64_t e = 0;
    auto advance = [&]() {                      // complete rounds: halting (node.ts:116-145 as DESIGN §2)
      while (full(S.comp + (cur & 3u) * 64u, S.killed)) {
        if (full(S.decided, S.killed)) { halted = 1; R = cur; return; }
        if (cur >= p.k_max) { halted = 2; R = cur; return; }
        if (lane < 64u) S.comp[(cur & 3u) * 64u + lane] = 0ull;
        ++cur;
      }
    };
    while (!halted) {
      // ---- scheduled GET /stop (node.ts:191-194) before delivery e
      bool crashed = false;
      while ((next_key >> 12) == e) {
        const uint32_t i = (uint32_t)(next_key & 4095u);
        if (lane == 0u) {
          S.killed[i >> 6] |= 1ull << (i & 63u);
          S.ibox[2u * i] |= kKilled;
          S.ibox[2u * i + 1u] |= kKilled;
        }
        crashed = true;
        if (kr) {
          for (uint32_t j = lane; j < kr; j += 64u)
            if (S.rstops[j] == next_key) S.rstops[j] = ~0ull;
          next_key = rstops_min();
        } else {
          ++next;
          next_key = next < p.ev_nstops ? p.ev_stops[next] : ~0ull;
        }
      }
      if (crashed) {
        wsync();
        const bool alive = lane < NWd && S.killed[lane] != allw;
        if (!__any(alive)) { halted = 3; break; }
        advance();
        if (halted) break;
      }
      if (len == 0u) { halted = 3; break; }
      // ---- a batch of speculative events e .. e + B - 1.  A small pool (a small
      // network) has a trigger every few deliveries and picks that collide, so
      // its batches are shorter: B <= max(8, len / 8) keeps the collision scan
      // and the replay up to a trigger short (any B gives the same result).
      const uint32_t bcap = len >> 3 > 8u ? len >> 3 : 8u;
      uint64_t B = len < 64u ? len : 64u;
      if (B > bcap) B = bcap;
      if (next_key != ~0ull) {
        const uint64_t until = (next_key >> 12) - e;
        if (until < B) B = until;
      }
      uint32_t pk = 0, pv = 0, tv = 0;
      // agent-scope loads are L2-served (no stale L1 line after the last batch's stores)
      auto load = [&](uint32_t i) { return __hip_atomic_load(&pool[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
      if (pf_e == e && pf_len == len && pf_b == B) {
        // the previous batch ran to its end: its prefetch is this batch, except
        // for the words that batch wrote after they were read (S.wrote marks
        // them by their low 16 bits; a false match only reloads)
        pk = pf_pk;
        pv = pf_pv;
        tv = pf_tv;
        bool stale = false;
        if (lane < B) {
          const uint32_t kq = pk & 0xFFFFu, kt = (len - 1u - lane) & 0xFFFFu;
          stale = ((S.wrote[kq >> 5] >> (kq & 31u)) & 1u) || ((S.wrote[kt >> 5] >> (kt & 31u)) & 1u);
        }
        if (stale) {
          pv = load(pk);
          tv = load(len - 1u - lane);
        }
      } else if (lane < B) {
        const uint64_t z = mix64(rng + (uint64_t)(lane + 1u) * kGamma);
        pk = (uint32_t)(((uint64_t)(uint32_t)(z >> 32) * (uint64_t)(len - lane)) >> 32);
        pv = load(pk);
        tv = load(len - 1u - lane);
      }
      if (wq != 0xFFFFFFFFu) S.wrote[(wq & 0xFFFFu) >> 5] = 0u;   // the previous batch's marks are spent
      wq = 0xFFFFFFFFu;
      // ---- prefetch: the next batch's picks and words, as if this batch runs to
      // its end without a trigger (no scheduled stop at its end)
      pf_e = ~0ull;
      {
        const uint32_t len2 = len - (uint32_t)B;
        const uint32_t bcap2 = len2 >> 3 > 8u ? len2 >> 3 : 8u;   // the same batch rule as above
        uint64_t B2 = len2 < 64u ? len2 : 64u;
        if (B2 > bcap2) B2 = bcap2;
        bool ok = len2 > 0u;
        if (next_key != ~0ull) {
          const uint64_t until2 = (next_key >> 12) - (e + B);
          if (until2 == 0u) ok = false;
          else if (until2 < B2) B2 = until2;
        }
        if (ok) {
          pf_e = e + B;
          pf_len = len2;
          pf_b = B2;
          if (lane < B2) {
            const uint64_t z = mix64(rng + (uint64_t)((uint32_t)B + lane + 1u) * kGamma);
            pf_pk = (uint32_t)(((uint64_t)(uint32_t)(z >> 32) * (uint64_t)(len2 - lane)) >> 32);
            pf_pv = load(pf_pk);
            pf_tv = load(len2 - 1u - lane);
          }
        }
      }
      // ---- the batch's messages.  Event i takes the message at q_i = pk and
      // moves the one at t_i = len - 1 - i there (swap-remove).  As the batch's
      // earlier events left the pool, position p holds the value moved by the
      // last event j < i with q_j = p, else the pool's own word.  So per lane:
      //   a = last j < i with q_j = q_i, b = last j < i with q_j = t_i (one scan
      //   over the batch's picks, no cross-iteration dependency);
      //   moved_i = moved_b (b exists) else pool[t_i] -- a chain i -> b -> ...
      //   resolved to its root by pointer jumping (6 bpermute steps for 64);
      //   msg_i = moved_a (a exists) else pool[q_i];
      // and event i's write is the position's last one iff no later event
      // of the batch picks q_i (nx = the first such j).
      // Usually no two picks of a batch share a position and no pick is one of
      // the batch's tail positions (~64^2 / len): a 64 K-bit LDS bitmap of the
      // picks' low 16 bits finds the batches that may have one (q-q or q-t key
      // collisions, ~10 % at len ~ 7·10^5 with false positives), and only those
      // run the scan.
      const uint32_t qi = pk, ti = len - 1u - lane;
      uint32_t a1 = 0u, b1 = 0u, nx = 64u;      // a + 1, b + 1 (0: none)
      uint32_t ovv = tv, mine = pv;             // moved_i, and the message event i delivers
      bool maybe = false;
      if (lane < B) {
        const uint32_t kq = qi & 0xFFFFu, kt = ti & 0xFFFFu;
        const uint32_t old = atomicOr(&S.picks[kq >> 5], 1u << (kq & 31u));
        maybe = (old >> (kq & 31u)) & 1u;
        asm volatile("" ::: "memory");           // the read below after every lane's mark (in-order LDS)
        maybe = maybe || ((S.picks[kt >> 5] >> (kt & 31u)) & 1u);
      }
      if (__any(maybe)) {
        for (uint32_t j = 0; j < (uint32_t)B; ++j) {
          const uint32_t qj = rl(pk, j);
          const uint32_t lt = below_mask(j, lane), gt = below_mask(lane, j);   // j < i, j > i
          const uint32_t eq_q = zero_mask(qj ^ qi), eq_t = zero_mask(qj ^ ti);
          a1 = umax(a1, eq_q & lt & (j + 1u));
          b1 = umax(b1, eq_t & lt & (j + 1u));
          nx = umin(nx, j | (~(eq_q & gt) & 64u));
        }
        uint32_t root = b1 ? b1 - 1u : lane;
        for (int step = 0; step < 6; ++step)
          root = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(root << 2), (int)root);
        ovv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(root << 2), (int)tv);
        const uint32_t via = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((a1 ? a1 - 1u : lane) << 2), (int)ovv);
        mine = a1 ? via : pv;
      }
      if (lane < B) S.picks[(qi & 0xFFFFu) >> 5] = 0u;   // the bitmap is empty again for the next batch
      // ---- POST /message (node.ts:45-158), all B deliveries at once: each
      // adds {len, c0 | c1} to its receiver's inbox slot unless the receiver is
      // killed (node.ts:45) or the round is beyond the oracle's window.  When
      // no slot reaches the quorum (node.ts:52, :88) inside the batch, that is
      // the sequential result (the adds commute); otherwise they are undone and
      // the batch is replayed one delivery at a time up to its first trigger.
      uint32_t used = (uint32_t)B, trig = 0xFFFFFFFFu, tmsg = 0u;
      uint64_t tbox = 0ull;
      {
        uint64_t inc = 0ull;
        uint64_t *bp = nullptr;
        if (lane < B) {
          const uint32_t to = mine & 4095u, ph = (mine >> 12) & 1u, xv = (mine >> 13) & 3u;
          const uint32_t k = cur + (((mine >> 15) - cur) & 3u);
          bp = &S.ibox[2u * to + ph];
          if (!(*bp & kKilled) && k < p.k_max + 3u)
            inc = (1ull << 26) + (xv == 0u ? 1ull : (xv == 1u ? 1ull << 13 : 0ull));
        }
        bool crossed = false;
        if (inc) {
          const uint64_t old = __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(bp), inc,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          crossed = ((old >> 26) & kC13) + 1u == quorum;
        }
        if (__any(crossed)) {
          if (inc)
            __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(bp), 0ull - inc, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
          __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the undo lands before the replay reads
          for (uint32_t i = 0; i < (uint32_t)B; ++i) {
            const uint32_t msg = rl(mine, i);
            const uint32_t to = msg & 4095u, ph = (msg >> 12) & 1u, xv = (msg >> 13) & 3u;
            const uint32_t k = cur + (((msg >> 15) - cur) & 3u);
            uint64_t *sp = &S.ibox[2u * to + ph];
            uint64_t b = *sp;
            if (b & kKilled) continue;             // node.ts:45
            if (k >= p.k_max + 3u) continue;        // beyond the oracle's round window
            b += 1ull << 26;                        // len
            if (xv == 0u) b += 1ull;                // c0
            else if (xv == 1u) b += 1ull << 13;     // c1
            if (((b >> 26) & kC13) != quorum) {     // node.ts:52, :88
              if (lane == 0u) *sp = b;
              continue;
            }
            if (lane == 0u) *sp = 0ull;             // every message of the phase arrived: the slot is free
            trig = i;
            tmsg = msg;
            tbox = b;
            used = i + 1u;
            break;
          }
        }
      }
      // ---- the batch's pool writes: each used event's, unless a later used
      // event overwrites its position or the position was popped
      if (lane < used && nx >= used && qi < len - used) {
        pool[qi] = ovv;
        atomicOr(&S.wrote[(qi & 0xFFFFu) >> 5], 1u << (qi & 31u));     // for the next batch's prefetch
        wq = qi;
      }
      len -= used;
      rng += (uint64_t)used * kGamma;
      e += used;
      if (trig == 0xFFFFFFFFu) {
        __threadfence_block();
        continue;
      }
      // ---- a trigger (node.ts:52-80 R-phase, :88-157 P-phase)
      const uint32_t to = tmsg & 4095u, ph = (tmsg >> 12) & 1u;
      const uint32_t k = cur + (((tmsg >> 15) - cur) & 3u);
      const uint32_t c0 = (uint32_t)(tbox & kC13), c1 = (uint32_t)((tbox >> 13) & kC13);
      uint32_t body;
      if (ph == 0u) {
        const uint32_t v = c0 > c1 ? 0u : (c1 > c0 ? 1u : 2u);
        body = (1u << 12) | (v << 13) | ((k & 3u) << 15);
      } else {
        int8_t nx;
        bool dec = true;
        if (c0 > F) nx = 0;
        else if (c1 > F) nx = 1;
        else {
          dec = false;
          if (c0 + c1 > 0u && c0 > c1) nx = 0;
          else if (c0 + c1 > 0u && c0 < c1) nx = 1;
          else {
            const uint32_t c = S.cidx[to];     // the coin of compact node c in round k (node.ts:111)
            const uint4 rr = coin_block<false>(k0, k1, tlo, thi, c, k);
            nx = (int8_t)((coin_word(rr, k) >> (c & 31u)) & 1u);
          }
        }
        if (lane == 0u) {
          S.xs[to] = nx;
          S.ks[to] = (int16_t)(k + 1u);
          if (dec) S.decided[to >> 6] |= 1ull << (to & 63u);
          S.comp[(k & 3u) * 64u + (to >> 6)] |= 1ull << (to & 63u);
        }
        wsync();
        advance();
        if (halted) break;
        body = ((uint32_t)(nx & 3) << 13) | (((k + 1u) & 3u) << 15);
      }
      if ((uint64_t)len + N > cap) { overflow = true; halted = 3; break; }
      __threadfence_block();
      for (uint32_t d = lane; d < N; d += 64u) pool[len + d] = d | body;
      len += N;
      __threadfence_block();
    }
    // ---- outcome over the nodes still running
    bool any0 = false, any1 = false, anyq = false, nl = false;
    wsync();
    for (uint32_t i = lane; i < N; i += 64u) {
      if ((S.killed[i >> 6] >> (i & 63u)) & 1ull) continue;
      nl = true;
      const int8_t v = S.xs[i];
      if (v == 0) any0 = true; else if (v == 1) any1 = true; else anyq = true;
    }
    const bool g0 = __any(any0), g1 = __any(any1), gq = __any(anyq), gl = __any(nl);
    const uint32_t v = (!gl || gq || (g0 && g1)) ? 2u : (g1 ? 1u : 0u);
    if (lane == 0u) {
      atomicAdd(&lhist[halted == 1u ? (R * 3u + v) : v], 1u);
      if (halted == 1u && v == 2u) atomicAdd(&lhist[p.hist_len - 1u], 1u);
      if (overflow && p.rounds_out) atomicOr(p.rounds_out, 0x80000000u);
      if (overflow && p.overflow) atomicOr(p.overflow, 2u);
      if (p.node_out && p.rounds_out) atomicOr(p.rounds_out, halted == 1u ? R : 0u);
    }
    if (p.node_out) {
      for (uint32_t i = lane; i < N; i += 64u) {
        bo_node_state ns;
        const bool f = S.ks[i] < 0 && S.xs[i] < 0;   // faulty from launch (never ran)
        ns.killed = (int8_t)((S.killed[i >> 6] >> (i & 63u)) & 1ull);
        ns.x = S.xs[i];
        ns.decided = f ? (int8_t)-1 : (int8_t)((S.decided[i >> 6] >> (i & 63u)) & 1ull);
        ns.pad = 0;
        ns.k = S.ks[i];
        p.node_out[i] = ns;
      }
    }
    wsync();
  }
  wsync();
  for (uint32_t i = lane; i < p.hist_len; i += 64u) {   // flush_hist
    const uint32_t c = lhist[i];
    if (c) atomicAdd(&p.hist[i], (unsigned long long)c);
  }
}

bool event_big_lds_pool(const KParams &p) { return (uint64_t)p.ev_cap * 4u <= kEventBigLdsPool; }

uint32_t event_big_lds_bytes(const KParams &p) {
  const uint32_t N = p.N;
  return p.hist_bytes + 16u * N + 8u * 64u * 6u + 2u * ((N + 3u) & ~3u) * 2u + ((N + 15u) & ~15u) + 2u * 2048u * 4u +
         8u * 64u + 8u * p.ev_rstops +   // random /stop schedule: Floyd set, keys
         (event_big_lds_pool(p) ? 4u * p.ev_cap : 0u);   // the message pool, when it fits
}

template <bool LP>
static hipError_t launch_event_big_lp(const KParams &p, int grid, hipStream_t s) {
  const uint32_t lds = event_big_lds_bytes(p);
  if (lds > 64u * 1024u) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&benor_event_big_kernel<LP>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(benor_event_big_kernel<LP>, dim3(grid), dim3(64), lds, s, p);
  return hipGetLastError();
}

hipError_t launch_event_big(const KParams &p, int grid, hipStream_t s) {
  if (p.live_box) return hipErrorInvalidValue;      // live runs are benor_event_live.hip's
  return event_big_lds_pool(p) ? launch_event_big_lp<true>(p, grid, s) : launch_event_big_lp<false>(p, grid, s);
}

}  // namespace benor
