// benor_event_live.hip -- the event kernels of live runs (r06): the default
// startConsensus (bo_consensus_start_live) and network starts with a /stop
// schedule, at every N <= 4096.
//
// The reference's GET /start answers before consensus finishes
// (consensus.ts:3-8, node.ts:167-188): its round loop is the POST /message
// handler (node.ts:43-163) firing message by message, and a GET /stop
// (node.ts:191-194) or GET /getState (node.ts:197-199) may arrive at any
// moment.  These kernels run the message-granular model of oracle (iii),
// oracle/benor_oracle.c event_trial() -- one delivery per event in the seeded
// order (uniform pick from the pending pool, swap-remove), scheduled and live
// stops applied before their delivery count -- for ONE trial per workgroup,
// in one of three forms by N (launch_event_wg):
//
//   * N > 64 (benor_event_wg_kernel): a control wave and up to 15 event
//     waves.  The event waves take a batch of B <= 64 W consecutive events:
//     lane i draws the pick of event e + i assuming no trigger (splitmix64 is
//     a counter), loads the two pool words its swap-remove touches, and
//     inserts its pick into an LDS hash table {position, pickers, first
//     picker}.  A word one earlier event of the batch moved is forwarded; a
//     second level, or a third picker of one position, cuts the batch there.
//     The deliveries are applied at once with 64-bit LDS adds of
//     {len, c0 | c1} to the receivers' inbox slots.  With exactly F faulty
//     every slot receives exactly N - F messages per round (each trigger fires
//     once), so a slot that reaches its quorum inside the batch
//     triggers at the LAST batch event into it; the batch ends after the
//     earliest such event and the later events' adds are undone.  The used
//     events write their moved words back, the control wave runs the trigger
//     (node.ts:53-80 R-phase, :89-157 P-phase: decide, adopt, coin,
//     all-decided halting) and the event waves append its broadcast of N
//     messages.  The control wave issues no pool access: it owns the round
//     state, applies scheduled and live /stop requests, and polls the
//     host-mapped mailbox with an uncached load that it consumes ~20 us later
//     (so the PCIe round trip is never waited for);
//   * 16 < N <= 64 (benor_event_wave_kernel): one wave, micro-batches of up to
//     64 events with the pool in LDS, every chain of the batch's moves
//     followed back, so a batch runs to its first trigger;
//   * N <= 16 (benor_event_reg_kernel): one wave, one event per step, the
//     pool, the inbox slots and the node state in registers.
//
// All three serve GET /getState snapshots: on request they write every node's
// {killed, x, decided, k} at a batch boundary to host memory with the
// delivery count it reflects, so a snapshot is oracle (iii) truncated at
// that count.
//
// Pool words (workgroup and LDS-wave forms): `to | ph << 12 | x << 13 |
// (k & 3) << 15` (k decoded against the completion round `cur`, as
// benor_event_big.hip), in HBM scratch or -- when 4N^2 + 64 words fit
// kEventBigLdsPool (N <= 78) -- in LDS.
#include "benor_device.h"

#include <type_traits>
#include <utility>

namespace benor {

namespace {

constexpr uint64_t kGm = 0x9E3779B97F4A7C15ull;   // splitmix64 increment
constexpr uint64_t kF13 = (1ull << 13) - 1ull;
constexpr uint64_t kDead = 1ull << 63;             // inbox slot of a killed node

__device__ __forceinline__ uint64_t smix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// LDS hash slots per batch (a power of two, KParams::ev_hs): four times the
// batch where LDS allows, else twice -- a wave's slowest lane probes about
// twice as far at load 1/2 as at 1/4, one LDS round trip per probe
constexpr uint32_t pow2_ceil(uint32_t v) { uint32_t r = 1u; while (r < v) r <<= 1; return r; }

// The control block: the round state the control wave publishes for the next
// batch, and the batch's reduction words (double-buffered by batch parity:
// the control wave prepares batch n + 1 while the event waves still read
// batch n's).
struct Ctl {
  uint64_t rng;        // splitmix64 state at the batch's first delivery
  uint64_t tbox;       // the first trigger's inbox slot {c0, c1, len} (its slot is then cleared)
  uint32_t len;        // pending messages
  uint32_t B;          // the batch's events
  uint32_t cur;        // completion round (decodes a message's k & 3)
  uint32_t halted;     // 0 running, 1 all decided, 2 k_max, 3 stall
  uint32_t snap;       // serve a snapshot before this batch (the request number), 0 none
  uint32_t body;       // the last batch's trigger broadcast, ~0 none
  uint32_t bpos;       // where it goes (the pool's length after that batch)
  uint32_t tmsg;       // the batch's first trigger message
  uint32_t overflow;
  uint32_t R;          // the halting round (after the run)
  uint32_t conf[2];    // first event of the batch that cannot be resolved (B if none)
  uint32_t ncross[2];  // inbox slots that reached their quorum in the batch
  uint32_t trig[2];    // the batch's first trigger event (~0: none)
};

// The mailbox poll's clock: shader cycles.  A poll is consumed >= 20 us
// after it was issued (its PCIe round trip is long done, so no wait): 48000
// cycles at 2.4 GHz, a slower clock only spaces the polls further.  Each
// consumed poll costs the batch loop ~500 cycles: at 5 us it was ~7 % of a live
// run at N = 1024 (10.6 against 9.85 ms with polls 1 ms apart,
// tools/live_profile.py); a GET /stop or /getState waits at most ~20 us more
// for the kernel, against the reference's HTTP round trip per request.
constexpr long long kPollCycles = 48000;
__device__ __forceinline__ long long poll_clock() { return (long long)__builtin_amdgcn_s_memtime(); }

__device__ __forceinline__ uint32_t hslot(uint32_t key, uint32_t mask) { return (key * 0x9E3779B1u >> 11) & mask; }

// A wave-uniform value read from LDS or global memory: the compiler cannot see
// that every lane read the same word, and left to itself turns the round
// state and everything it controls into exec-masked vector code.
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return (uint64_t)uni((uint32_t)v) | ((uint64_t)uni((uint32_t)(v >> 32)) << 32);
}

}  // namespace

// Wave 0: control.  Waves 1..W: events, one per lane.  One trial per
// workgroup (grid-stride over the launch's trials).
//
// A batch of B events e .. e + B - 1 (lane i: event e + i) in four phases
// between workgroup barriers:
//   1. pick q_i (assuming no trigger), load pool[q_i] and the tail word
//      pool[t_i], t_i = len - 1 - i; count the batch's pickers of q_i in an
//      LDS hash slot {position, count, first picker}; a pick of a tail
//      position names the later event whose tail it overwrites (bmax);
//   2. resolve, one level deep: event i's message is pool[q_i] unless an
//      earlier event a picked q_i (then the word a moved there), and the word
//      it moves is pool[t_i] unless an earlier event b picked t_i (then the
//      word b moved).  A second level (the moved word was itself forwarded),
//      or a third picker of one position, cuts the batch before that event;
//   3. deliver the uncut prefix at once (64-bit LDS adds of {len, c0 | c1});
//      a slot that reaches its quorum triggers at its last batch event, and
//      the batch ends after the earliest one (later adds undone);
//   4. each position's last writer among the used events stores its moved
//      word (unless the position was popped).
// Meanwhile the control wave runs the trigger, applies the next batch's
// scheduled and live stops, serves snapshot requests and publishes the next
// batch; the event waves then append the trigger's broadcast.
template <int W, bool LP, bool ST>
__global__ void __launch_bounds__(64 * (W + 1)) benor_event_wg_kernel(KParams p) {
  constexpr uint32_t T = 64u * (uint32_t)W;        // event lanes
  const uint32_t HS = p.ev_hs;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const bool ctl = tid < 64u;                      // the control wave
  const uint32_t ei = tid - 64u;                   // event lane index (event waves)
  const uint32_t N = p.N, F = p.F, quorum = p.N - p.F, m = p.m;
  const uint32_t NWd = (N + 63u) >> 6;
  Ctl &C = *reinterpret_cast<Ctl *>(smem);
  unsigned char *q = smem + ((sizeof(Ctl) + 15u) & ~15u);
  uint64_t *ibox = reinterpret_cast<uint64_t *>(q);               // [2N] {c0, c1, len}, bit 63 killed
  uint64_t *killed = ibox + 2u * N;                              // [64]
  uint64_t *decided = killed + 64;                               // [64]
  uint64_t *comp = decided + 64;                                 // [4][64] round k complete at k & 3
  uint64_t *ht = comp + 256;                                     // [HS] (pos + 1) << 32 | pickers << 16 | first
  uint64_t *rset = ht + HS;                                      // [64] random /stop schedule: Floyd set
  uint64_t *rstops = rset + 64;                                  // [ev_rstops] (event << 12 | node), ~0 applied
  uint32_t *smax = reinterpret_cast<uint32_t *>(rstops + p.ev_rstops);   // [2N] last batch event + 1 into a crossed slot
  uint32_t *bmax = smax + 2u * N;                                // [T] last earlier event + 1 that picked t_i
  uint32_t *nxt = bmax + T;                                      // [T] the second picker + 1 of q_i (first picker's entry)
  uint32_t *tvs = nxt + T;                                       // [T] the tail words
  int16_t *ks = reinterpret_cast<int16_t *>(tvs + T);            // [N]
  uint16_t *cidx = reinterpret_cast<uint16_t *>(ks + ((N + 7u) & ~7u));  // [N] compact index (coins)
  int8_t *xs = reinterpret_cast<int8_t *>(cidx + ((N + 7u) & ~7u));       // [N]
  uint32_t *pool;
  if constexpr (LP) pool = reinterpret_cast<uint32_t *>(xs + ((N + 15u) & ~15u));
  else pool = p.scratch + (uint64_t)blockIdx.x * p.ev_stride;
  const uint32_t cap = p.ev_cap;
  const uint64_t allw = lane < NWd ? (N >= 64u * (lane + 1u) ? ~0ull : (1ull << (N - 64u * lane)) - 1ull) : 0ull;
  const uint64_t wmask = NWd >= 64u ? ~0ull : ((1ull << NWd) - 1ull);
  const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
  uint32_t *box = p.live_box;                                    // host-mapped mailbox (live runs)

  // a | b == all, over the bitset words (control wave: one word per lane)
  auto full = [&](const uint64_t *a, const uint64_t *b) {
    const bool ok = lane >= NWd || ((a[lane] | b[lane]) == allw);
    return (__ballot(ok) & wmask) == wmask;
  };
  // pool words: only this workgroup (one CU) reads and writes its slice, so
  // workgroup-scope loads, served by the CU's L1 and its XCD's L2 (an
  // agent-scope load bypasses the L2 -- not coherent across XCDs -- and went to
  // MALL/HBM, tools/live_profile.py); every pool store is drained (vm_drain)
  // before the barrier that orders it with another wave's load
  auto load = [&](uint32_t i) -> uint32_t {
    if constexpr (LP) return pool[i];
    else return __hip_atomic_load(&pool[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  auto vm_drain = [&]() {
    if constexpr (!LP) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
  };

  for (uint32_t i = tid; i < HS; i += blockDim.x) ht[i] = 0ull;
  for (uint32_t i = tid; i < 2u * N; i += blockDim.x) smax[i] = 0u;
  for (uint32_t i = tid; i < T; i += blockDim.x) {
    bmax[i] = 0u;
    nxt[i] = 0u;
  }

  // the control wave's mailbox poll: lane l < NWd reads request bits 64l ..
  // 64l + 63, lane 0 also the request sequence word and lane 1 the snapshot
  // request; issued at `polled`, consumed >= kPollCycles later.  The host sets a
  // burst's bits (stopConsensus: every node) and then bumps the sequence word,
  // so the bits of the poll AFTER the one that saw the new sequence hold the
  // whole burst, which then lands at one delivery count.
  uint64_t pv_req = 0ull;
  uint32_t pv_word = 0u, snap_served = 0u, seq_seen = 0u;
  bool apply_next = false;
  long long polled = 0;
  bool poll_out = false;
  auto poll_issue = [&]() {
    if (lane < NWd)
      pv_req = __hip_atomic_load(reinterpret_cast<uint64_t *>(box + kLiveReq) + lane, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 0u) pv_word = __hip_atomic_load(box, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 1u) pv_word = __hip_atomic_load(box + kSnapReq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    polled = poll_clock();
    poll_out = true;
  };
  if (ctl && box) poll_issue();

  for (uint64_t t = blockIdx.x; t < p.trial_count; t += gridDim.x) {
    const uint64_t trial = p.trial_begin + t;
    const uint32_t tlo = (uint32_t)trial, thi = (uint32_t)(trial >> 32);
    // ---- node.ts:21-26: faulty nodes killed, live nodes x = initial value
    if (ctl) {
      killed[lane] = lane < NWd ? allw : 0ull;     // every node, then the live ones cleared
      decided[lane] = 0ull;
      for (int r = 0; r < 4; ++r) comp[r * 64 + lane] = 0ull;
    }
    for (uint32_t i = tid; i < N; i += blockDim.x) {
      xs[i] = -1;
      ks[i] = -1;
      ibox[2u * i] = kDead;
      ibox[2u * i + 1u] = kDead;
    }
    __syncthreads();
    for (uint32_t c = tid; c < m; c += blockDim.x) {
      const uint32_t i = p.live_ids[c];
      int8_t v;
      if (p.init_mode == BO_INIT_RANDOM) {        // oracle_random_init
        if (m <= 32u) {
          v = (int8_t)((init_word_small(k0, k1, trial) >> c) & 1u);
        } else {
          const uint4 ir = philox4x32_10<false>(k0, k1, make_uint4(tlo, thi, c >> 7, kStreamInit << 24));
          v = (int8_t)((coin_word_v(ir, ((c >> 5) & 3u) + 1u) >> (c & 31u)) & 1u);
        }
      } else {
        v = p.init_x[i];
      }
      xs[i] = v;
      ks[i] = 1;                                   // /start: k = 1 (node.ts:172)
      cidx[i] = (uint16_t)c;
      ibox[2u * i] = 0ull;
      ibox[2u * i + 1u] = 0ull;
      __hip_atomic_fetch_and(reinterpret_cast<unsigned long long *>(&killed[i >> 6]), ~(1ull << (i & 63u)),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    // ---- /start (node.ts:167-188): every live node broadcasts its x, in node order
    if (!ctl) {
      for (uint32_t c = 0; c < m; ++c) {
        const uint32_t body = ((uint32_t)(xs[p.live_ids[c]] & 3) << 13) | (1u << 15);
        for (uint32_t to = ei; to < N; to += T) pool[c * N + to] = to | body;
      }
      vm_drain();
    }
    // ---- the /stop schedule: explicit (ev_stops, ascending event << 12 | node)
    // or random (crash_count): Floyd over compact live indices from Philox
    // stream 4, then one uniform delivery count in [0, crash_window) per pick
    const uint32_t kr = p.ev_rstops;
    if (ctl && kr) {
      rset[lane] = 0ull;
      __builtin_amdgcn_wave_barrier();
      if (lane == 0u) {
        DStream ds;
        ds.k0 = k0; ds.k1 = k1; ds.c0 = tlo; ds.c1 = thi; ds.c2 = 0u; ds.c3 = kStreamCrash << 24; ds.widx = 0;
        ds.sh = 12u;
        for (uint32_t j = m - kr, n = 0; j < m; ++j, ++n) {
          const uint32_t tt = ds.uniform(j + 1u);
          const uint32_t idx = ((rset[tt >> 6] >> (tt & 63u)) & 1ull) ? j : tt;
          rset[idx >> 6] |= 1ull << (idx & 63u);
          rstops[n] = idx;
        }
        for (uint32_t n = 0; n < kr; ++n) {
          const uint32_t when = ds.uniform(p.crash_window);
          rstops[n] = ((uint64_t)when << 12) | p.live_ids[(uint32_t)rstops[n]];
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    }
    auto rstops_min = [&]() {                      // control wave: the random schedule's next key
      uint64_t v = ~0ull;
      for (uint32_t i = lane; i < kr; i += 64u) v = v < rstops[i] ? v : rstops[i];
      for (int off = 32; off >= 1; off >>= 1) {
        const uint64_t o = __shfl_xor(v, off);
        v = v < o ? v : o;
      }
      return v;
    };
    // control wave: round completion and halting (node.ts:116-145 as DESIGN §2)
    auto advance = [&](uint32_t &cur, uint32_t &halted, uint32_t &R) {
      while (full(comp + (cur & 3u) * 64u, killed)) {
        if (full(decided, killed)) { halted = 1u; R = cur; return; }
        if (cur >= p.k_max) { halted = 2u; R = cur; return; }
        comp[(cur & 3u) * 64u + lane] = 0ull;
        ++cur;
      }
    };

    // The batch loop, as two loops that meet at the same barriers (H B C
    // D [E F G] per batch): the control wave's and the event waves'.  Kept
    // apart so that the control wave's in-flight mailbox poll is never waited
    // for by an s_waitcnt the event code needs.
    if (ctl) {
      // diagnostics (BENOR_EVENT_STATS): batch counters and the shader cycles
      // between the control wave's barriers, accumulated per trial
      unsigned long long *const stats = ST ? p.ev_stats : nullptr;   // ST: compiled in only for BENOR_EVENT_STATS
      uint64_t st[24] = {};
      uint64_t t_prev = stats ? __builtin_amdgcn_s_memtime() : 0ull;
      const uint64_t t_start = t_prev, w_start = stats ? (uint64_t)wall_clock64() : 0ull;
      auto stamp = [&](int slot) {
        if (stats) {
          const uint64_t t = __builtin_amdgcn_s_memtime();
          st[slot] += t - t_prev;
          t_prev = t;
        }
      };
      uint32_t next = 0;
      uint64_t next_key = uni64(kr ? rstops_min() : (p.ev_nstops ? p.ev_stops[0] : ~0ull));
      uint64_t e = 0, rng;
      {
        const uint4 o = philox4x32_10<false>(k0, k1, make_uint4(tlo, thi, 0u, kStreamOrder << 24));
        rng = (((uint64_t)o.x << 32) | o.y) ^ 0xD1B54A32D192ED03ull;
      }
      uint32_t len = m * N, cur = 1u, R = 0u, halted = 0u, body = 0xFFFFFFFFu, par = 0u, overflow = 0u;
      // ---- the next batch, at delivery e: scheduled and live GET /stop
      // (node.ts:191-194) before delivery e, a snapshot request, halting, its size
      auto prepare = [&]() {
        bool crashed = false;
        while ((next_key >> 12) == e) {
          const uint32_t i = (uint32_t)(next_key & 4095u);
          if (lane == 0u) {
            killed[i >> 6] |= 1ull << (i & 63u);
            ibox[2u * i] |= kDead;
            ibox[2u * i + 1u] |= kDead;
          }
          crashed = true;
          if (kr) {
            for (uint32_t j = lane; j < kr; j += 64u)
              if (rstops[j] == next_key) rstops[j] = ~0ull;
            next_key = uni64(rstops_min());
          } else {
            ++next;
            next_key = uni64(next < p.ev_nstops ? p.ev_stops[next] : ~0ull);
          }
        }
        uint32_t snap = 0u;
        if (box && poll_out && poll_clock() - polled >= kPollCycles) {
          // live GET /stop requests and /getState snapshot requests: the poll
          // issued >= 20 us ago (its PCIe round trip is long done)
          const uint64_t req = apply_next ? pv_req : 0ull;   // a burst is complete one poll after its sequence
          const uint32_t seq = uni(__shfl(pv_word, 0)), sreq = uni(__shfl(pv_word, 1));   // uniform: keeps the loop scalar
          apply_next = seq != seq_seen;
          seq_seen = seq;
          uint64_t fresh = 0ull;
          if (lane < NWd) {
            fresh = req & allw & ~killed[lane];
            killed[lane] |= fresh;
          }
          for (uint64_t f = fresh; f; f &= f - 1ull) {
            const uint32_t i = 64u * lane + (uint32_t)__builtin_ctzll(f);
            ibox[2u * i] |= kDead;
            ibox[2u * i + 1u] |= kDead;
            __hip_atomic_store(box + kLiveEv + i, e < 0xFFFFFFFFull ? (uint32_t)e : 0xFFFFFFFEu, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
          }
          crashed = crashed || __any(fresh != 0ull);
          if (sreq != snap_served) {
            snap_served = sreq;
            snap = sreq;
          }
          poll_issue();
        }
        if (crashed) {
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
          const bool alive = lane < NWd && killed[lane] != allw;
          if (!__any(alive)) halted = 3u;
          else advance(cur, halted, R);
        }
        if (!halted && len == 0u) halted = 3u;
        uint32_t B = len < T ? len : T;
        if (next_key != ~0ull) {
          const uint64_t until = (next_key >> 12) - e;
          if (until < B) B = (uint32_t)until;
        }
        if (snap && !halted && lane == 0u) {       // the delivery count this snapshot reflects
          __hip_atomic_store(box + kSnapE, (uint32_t)e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(box + kSnapE + 1u, (uint32_t)(e >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return std::make_pair(B, halted ? 0u : snap);
      };
      auto publish = [&](uint32_t B, uint32_t snap, uint32_t bpos) {
        if (lane == 0u) {
          C.rng = rng;
          C.len = len;
          C.B = B;
          C.cur = cur;
          C.halted = halted;
          C.snap = snap;
          C.body = body;
          C.bpos = bpos;
          C.conf[par] = B;
          C.ncross[par] = 0u;
          C.trig[par] = 0xFFFFFFFFu;
        }
      };
      {
        const auto bs = prepare();
        publish(bs.first, bs.second, 0u);
      }
      uint32_t snap = 0u;
      for (;;) {
        // the loop-carried round state is wave-uniform; said so, the loop stays
        // scalar code (the compiler cannot prove it through the LDS reads)
        e = uni64(e);
        rng = uni64(rng);
        next_key = uni64(next_key);
        len = uni(len);
        cur = uni(cur);
        halted = uni(halted);
        body = uni(body);
        par = uni(par);
        next = uni(next);
        polled = (long long)uni64((uint64_t)polled);
        seq_seen = uni(seq_seen);
        snap_served = uni(snap_served);
        apply_next = uni(apply_next ? 1u : 0u) != 0u;
        poll_out = uni(poll_out ? 1u : 0u) != 0u;
        stamp(5);
        __syncthreads();                           // ---- H: the batch is published
        snap = uni(C.snap);
        const uint32_t B = uni(C.B);
        if (halted) break;
        stamp(11);
        __syncthreads();                           // ---- B: picks and loads
        stamp(6);
        if (snap && lane == 0u)                    // the snapshot's states are written
          __hip_atomic_store(box + kSnapSeq, snap, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        __syncthreads();                           // ---- C: resolution
        stamp(7);
        const uint32_t used0 = uni(C.conf[par]);
        __syncthreads();                           // ---- D: deliveries
        stamp(8);
        uint32_t used = used0;
        if (uni(C.ncross[par])) {
          __syncthreads();                         // ---- E
          __syncthreads();                         // ---- F
          used = uni(C.trig[par]) + 1u;
          __syncthreads();                         // ---- G
          stamp(9);
          st[14] += 1u;
        }
        if (stats) {
          st[0] += 1u;
          st[1] += used;
          st[2] += B;
          st[4] += used0 < B ? 1u : 0u;
          st[15] += snap ? 1u : 0u;
        }
        // read together: the trigger's message and slot (written by its event lane)
        const uint32_t tr = uni(C.trig[par]), tmsg_w = C.tmsg;
        const uint64_t tbox_w = C.tbox;
        body = 0xFFFFFFFFu;
        if (tr != 0xFFFFFFFFu) {
          // ---- the trigger (node.ts:52-80 R-phase, :88-157 P-phase)
          st[3] += 1u;
          const uint32_t tmsg = uni(tmsg_w);
          const uint32_t to = tmsg & 4095u, ph = (tmsg >> 12) & 1u;
          const uint32_t k = cur + (((tmsg >> 15) - cur) & 3u);
          const uint64_t tbox = uni64(tbox_w);
          const uint32_t c0 = (uint32_t)(tbox & kF13), c1 = (uint32_t)((tbox >> 13) & kF13);
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
                const uint32_t c = uni(cidx[to]);  // the coin of compact node c in round k (node.ts:111)
                const uint4 rr = coin_block<false>(k0, k1, tlo, thi, c, k);
                nx = (int8_t)uni((coin_word(rr, k) >> (c & 31u)) & 1u);
              }
            }
            if (lane == 0u) {
              xs[to] = nx;
              ks[to] = (int16_t)(k + 1u);
              if (dec) decided[to >> 6] |= 1ull << (to & 63u);
              comp[(k & 3u) * 64u + (to >> 6)] |= 1ull << (to & 63u);
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
            advance(cur, halted, R);
            if (!halted) body = ((uint32_t)(nx & 3) << 13) | (((k + 1u) & 3u) << 15);
          }
          if (body != 0xFFFFFFFFu && (uint64_t)(len - used) + N > cap) {
            body = 0xFFFFFFFFu;                    // the pool would overflow: stop (flagged)
            halted = 3u;
            overflow = 1u;
          }
        }
        stamp(21);
        body = uni(body);                          // uniform (see the loop head)
        halted = uni(halted);
        cur = uni(cur);
        const uint32_t bpos = len - used;
        len = bpos + (body != 0xFFFFFFFFu ? N : 0u);
        e += used;
        rng += (uint64_t)used * kGm;
        par ^= 1u;
        uint32_t nB = 0u, nsnap = 0u;
        if (!halted) {                             // (a halting trigger ends the run at once, as oracle (iii))
          const auto bs = prepare();
          nB = bs.first;
          nsnap = bs.second;
        }
        stamp(22);
        publish(nB, nsnap, bpos);
        stamp(10);
      }
      if (lane == 0u) {
        C.R = R;
        C.overflow = overflow;
      }
      if (stats && lane == 0u) {
        st[12] = __builtin_amdgcn_s_memtime() - t_start;
        st[13] = (uint64_t)wall_clock64() - w_start;
        for (int i = 0; i < 16; ++i) atomicAdd(&stats[i], (unsigned long long)st[i]);
        atomicAdd(&stats[21], (unsigned long long)st[21]);
        atomicAdd(&stats[22], (unsigned long long)st[22]);
      }
    } else {
      uint32_t par = 0u;
      // diagnostics (BENOR_EVENT_STATS): the first event wave's phase 1 split
      // into its own work and the wait for its pool words, and its phase 4
      unsigned long long *const stats = ST && tid == 64u ? p.ev_stats : nullptr;
      uint64_t s_work = 0ull, s_wait = 0ull, s_write = 0ull, s_pre = 0ull, s_drain = 0ull;
      for (;;) {
        __syncthreads();                           // ---- H
        const uint64_t t0 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
        // the last trigger's broadcast (node.ts:72-80, :149-157) goes to [bpos,
        // len): stored now, drained with this batch's loads; this batch itself
        // reads that region's words as they are, d | body for position bpos + d
        const uint32_t body = uni(C.body), bpos = uni(C.bpos);
        const bool fresh = body != 0xFFFFFFFFu;
        if (fresh)
          for (uint32_t d = ei; d < N; d += T) pool[bpos + d] = d | body;
        const uint32_t halted = uni(C.halted), B = uni(C.B), len = uni(C.len), cur = uni(C.cur), snap = uni(C.snap);
        const uint64_t rng = uni64(C.rng);
        if (halted) break;
        if (snap) {
          // GET /getState (node.ts:197-199) mid-run: every node's state as of
          // this batch's first delivery, to host memory (bo_get_states reads it
          // after the sequence word)
          for (uint32_t i = ei; i < N; i += T) {
            const bool f = ks[i] < 0 && xs[i] < 0;   // faulty from launch (never ran)
            const uint32_t kl =
                (uint32_t)(uint8_t)((killed[i >> 6] >> (i & 63u)) & 1ull) | ((uint32_t)(uint8_t)xs[i] << 8) |
                ((uint32_t)(uint8_t)(f ? (int8_t)-1 : (int8_t)((decided[i >> 6] >> (i & 63u)) & 1ull)) << 16);
            __hip_atomic_store(box + kSnapSt + 2u * i, kl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(box + kSnapSt + 2u * i + 1u, (uint32_t)(int32_t)ks[i], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
          }
          __builtin_amdgcn_s_waitcnt(0x0F70);      // vmcnt(0): the states reached the host
        }
        // ================= 1. picks: event e + i takes position q_i and moves
        // the word at t_i = len - 1 - i there (swap-remove)
        uint32_t qi = 0u, ti = 0u, pv = 0u, tv = 0u, hs = 0u;
        const bool act = ei < B;
        const uint64_t t1 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
        if (stats) s_pre += t1 - t0;
        if (act) {
          const uint64_t z = smix(rng + (uint64_t)(ei + 1u) * kGm);
          qi = (uint32_t)(((uint64_t)(uint32_t)(z >> 32) * (uint64_t)(len - ei)) >> 32);
          ti = len - 1u - ei;
          pv = fresh && qi >= bpos ? (qi - bpos) | body : load(qi);
          tv = fresh && ti >= bpos ? (ti - bpos) | body : load(ti);
          // the batch's pickers of qi: count and first (event index)
          const uint64_t key = (uint64_t)(qi + 1u) << 32;
          hs = hslot(qi, HS - 1u);
          for (;;) {
            uint64_t old = atomicCAS(reinterpret_cast<unsigned long long *>(&ht[hs]), 0ull, key | (1u << 16) | ei);
            if (old == 0ull) break;
            if ((old >> 32) == (key >> 32)) {      // a repeated pick (rare): count it, keep the first
              for (;;) {
                const uint64_t lo = old & 0xFFFFull;
                const uint64_t nv = (old & ~0xFFFFull) + (1ull << 16) | (lo < ei ? lo : (uint64_t)ei);
                const uint64_t r = atomicCAS(reinterpret_cast<unsigned long long *>(&ht[hs]), old, nv);
                if (r == old) break;
                old = r;
              }
              break;
            }
            hs = (hs + 1u) & (HS - 1u);
          }
          // a pick of a tail position overwrites the word a later event moves
          if (qi >= len - B && qi != ti) atomicMax(&bmax[len - 1u - qi], ei + 1u);
          if (stats) {
            const uint64_t t2 = __builtin_amdgcn_s_memtime();
            s_work += t2 - t1;
            __builtin_amdgcn_s_waitcnt(0x0F70);
            s_wait += __builtin_amdgcn_s_memtime() - t2;
          }
          tvs[ei] = tv;
        }
        const uint64_t t3 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
        vm_drain();                                // the broadcast's stores too, before any phase-4 store
        if (stats) s_drain += __builtin_amdgcn_s_memtime() - t3;
        __syncthreads();                           // ---- B
        // ================= 2. resolution, one level deep
        uint32_t msg = pv, moved = tv;
        if (act) {
          bool cut = false;
          const uint32_t b = bmax[ei];
          if (b) {                                 // t_i was overwritten by event b - 1: its moved word
            const uint32_t bb = bmax[b - 1u];
            if (bb) cut = true;
            else moved = tvs[b - 1u];
          }
          const uint64_t h = ht[hs];
          const uint32_t cnt = (uint32_t)(h >> 16) & 0xFFFFu, first = (uint32_t)h & 0xFFFFu;
          if (first != ei) {
            if (cnt >= 3u) cut = true;             // its earlier picker is not known: cut before it
            else {                                 // q_i was written by event `first`: its moved word
              nxt[first] = ei + 1u;
              const uint32_t ba = bmax[first];
              if (!ba) msg = tvs[first];
              else if (bmax[ba - 1u]) cut = true;
              else msg = tvs[ba - 1u];
            }
          }
          if (cut) atomicMin(&C.conf[par], ei);
        }
        __syncthreads();                           // ---- C
        const uint32_t used0 = uni(C.conf[par]);
        // ================= 3. POST /message (node.ts:45-158): the prefix's deliveries at once
        uint64_t inc = 0ull;
        uint32_t slot = 0u;
        if (act && ei < used0) {
          const uint32_t to = msg & 4095u, ph = (msg >> 12) & 1u, xv = (msg >> 13) & 3u;
          const uint32_t k = cur + (((msg >> 15) - cur) & 3u);
          slot = 2u * to + ph;
          if (k < p.k_max + 3u)                    // beyond the oracle's round window: dropped
            inc = (1ull << 26) + (xv == 0u ? 1ull : (xv == 1u ? 1ull << 13 : 0ull));
          if (inc) {
            const uint64_t old = __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(&ibox[slot]), inc,
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            // killed receivers drop the message (node.ts:45): their slot counts
            // on, never tested; a live slot crosses its quorum (node.ts:52, :88)
            if (!(old & kDead) && ((old >> 26) & kF13) + 1u == quorum) atomicAdd(&C.ncross[par], 1u);
          }
        }
        __syncthreads();                           // ---- D
        uint32_t used = used0;
        if (uni(C.ncross[par])) {
          // a crossed slot triggers at the last batch event into it; the batch
          // ends after the earliest such event
          bool mine = false;
          if (inc) {
            const uint64_t b = ibox[slot];
            mine = !(b & kDead) && ((b >> 26) & kF13) == quorum;
            if (mine) atomicMax(&smax[slot], ei + 1u);
          }
          __syncthreads();                         // ---- E
          if (mine) atomicMin(&C.trig[par], smax[slot] - 1u);
          __syncthreads();                         // ---- F
          const uint32_t tr = uni(C.trig[par]);
          if (mine) smax[slot] = 0u;
          if (inc && ei > tr)
            __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(&ibox[slot]), 0ull - inc,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (act && ei == tr) {
            // the trigger's slot is final (no later batch event goes there):
            // its counts to the control wave, and every message of the phase
            // arrived, so the slot is free
            C.tmsg = msg;
            C.tbox = ibox[slot];
            ibox[slot] = 0ull;
          }
          used = tr + 1u;
          __syncthreads();                         // ---- G
        }
        // ================= 4. pool writes: a position's last writer among the
        // used events stores its moved word, unless the position was popped
        const uint64_t t4 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
        if (act) {
          const uint32_t nx = nxt[ei];
          if (ei < used && (nx == 0u || nx - 1u >= used) && qi < len - used) pool[qi] = moved;
          ht[hs] = 0ull;                           // the tables are empty again for the next batch
          bmax[ei] = 0u;
          nxt[ei] = 0u;
        }
        vm_drain();
        if (stats) s_write += __builtin_amdgcn_s_memtime() - t4;
        par ^= 1u;
      }
      if (stats) {
        atomicAdd(&stats[16], (unsigned long long)s_work);
        atomicAdd(&stats[17], (unsigned long long)s_wait);
        atomicAdd(&stats[18], (unsigned long long)s_write);
        atomicAdd(&stats[19], (unsigned long long)s_pre);
        atomicAdd(&stats[20], (unsigned long long)s_drain);
      }
    }
    // ---- outcome over the nodes still running
    __syncthreads();
    const uint32_t hlt = C.halted, R = C.R;
    if (ctl) {
      bool any0 = false, any1 = false, anyq = false, nl = false;
      for (uint32_t i = lane; i < N; i += 64u) {
        if ((killed[i >> 6] >> (i & 63u)) & 1ull) continue;
        nl = true;
        const int8_t v = xs[i];
        if (v == 0) any0 = true; else if (v == 1) any1 = true; else anyq = true;
      }
      const bool g0 = __any(any0), g1 = __any(any1), gq = __any(anyq), gl = __any(nl);
      const uint32_t v = (!gl || gq || (g0 && g1)) ? 2u : (g1 ? 1u : 0u);
      if (lane == 0u) {
        atomicAdd(&p.hist[hlt == 1u ? (R * 3u + v) : v], 1ull);
        if (hlt == 1u && v == 2u) atomicAdd(&p.hist[p.hist_len - 1u], 1ull);
        if (C.overflow && p.rounds_out) atomicOr(p.rounds_out, 0x80000000u);
        if (C.overflow && p.overflow) atomicOr(p.overflow, 2u);
        if (p.node_out && p.rounds_out) atomicOr(p.rounds_out, hlt == 1u ? R : 0u);
      }
    }
    if (p.node_out) {
      for (uint32_t i = tid; i < N; i += blockDim.x) {
        bo_node_state ns;
        const bool f = ks[i] < 0 && xs[i] < 0;
        ns.killed = (int8_t)((killed[i >> 6] >> (i & 63u)) & 1ull);
        ns.x = xs[i];
        ns.decided = f ? (int8_t)-1 : (int8_t)((decided[i >> 6] >> (i & 63u)) & 1ull);
        ns.pad = 0;
        ns.k = ks[i];
        p.node_out[i] = ns;
      }
    }
    __syncthreads();
  }
  // the control wave's last poll must land before the wave ends
  if (ctl && box && poll_out) __builtin_amdgcn_s_waitcnt(0x0F70);
}

// ---------------------------------------------------------------------------
// Small networks (N <= kEventWaveMaxN): one wave, no barriers.  A batch of
// the workgroup kernel is cut by pick conflicts after ~sqrt(len) events, and
// at N = 10 the pool holds ~50 messages: its batches carried ~5 events for
// ~6k cycles, and a one-event-per-step loop costs ~700 cycles per event (one
// wave issues an instruction every ~10 cycles, tools/live_profile.py).  Here
// the wave takes micro-batches of up to 64 events, lane i = event e + i:
//   * picks as the workgroup kernel (they depend on e and len only), the pool
//     (4N^2 + 64 words) in LDS;
//   * no conflict cuts: the word event i takes is followed back through the
//     batch's earlier moves (position p before event i holds what the last
//     earlier event j with q_j = p moved there from t_j, before j; an LDS
//     table of 64-bit lane masks by position hash finds j), so a batch runs
//     to its first trigger;
//   * the batch is delivered at once (64-bit LDS adds of {len, c0 | c1} to
//     the inbox slots; a slot reaching its quorum triggers at its last batch
//     event, found by one ballot per crossed slot), later adds undone;
//   * each position the batch wrote and the pool keeps gets its last
//     writer's word, followed back the same way;
//   * the trigger (node.ts:52-80, :88-157), the stops, the mailbox and the
//     snapshots are scalar code, node state in lane registers (lane = node).
// The same definition as oracle (iii) event_trial() and the workgroup kernel.
template <bool ST>
__global__ void __launch_bounds__(64) benor_event_wave_kernel(KParams p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t pool[];   // [cap] messages | picks | writers | ibox | comp
  const uint32_t lane = threadIdx.x;
  const uint32_t N = p.N, F = p.F, quorum = p.N - p.F, m = p.m, kmax = p.k_max, cap = p.ev_cap;
  const uint32_t capa = (cap + 1u) & ~1u;
  uint32_t *qarr = pool + capa;                                      // [64] the batch's picks
  uint64_t *wm = reinterpret_cast<uint64_t *>(qarr + 64);            // [256] batch lanes writing a position, by hash
  uint64_t *ibox = wm + 256;                                         // [2N] {c0, c1, len}, bit 63 killed
  uint64_t *comp = ibox + 128;                                       // [4] round k complete at k & 3
  const uint64_t all = N >= 64u ? ~0ull : (1ull << N) - 1ull;
  const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
  uint32_t *box = p.live_box;
  unsigned long long *const stats = ST ? p.ev_stats : nullptr;   // ST: only for BENOR_EVENT_STATS
  // the mailbox poll, issued and consumed >= kPollCycles apart (as the
  // workgroup kernel's control wave): the wave waits for no PCIe round trip
  uint64_t pv_req = 0ull;
  uint32_t pv_word = 0u, snap_served = 0u, seq_seen = 0u;
  bool apply_next = false;
  long long polled = 0;
  auto poll_issue = [&]() {
    if (lane == 0u) pv_req = __hip_atomic_load(reinterpret_cast<uint64_t *>(box + kLiveReq), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 1u) pv_word = __hip_atomic_load(box, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 2u) pv_word = __hip_atomic_load(box + kSnapReq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    polled = poll_clock();
  };
  if (box) poll_issue();
  auto rl = [](uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); };
  auto wl = [lane](uint32_t v, uint32_t val, uint32_t l) { return lane == l ? val : v; };   // lane l of v := val
  auto lds_order = []() {                          // one wave's LDS operations are in order: compiler ordering only
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  };
  for (uint32_t i = lane; i < 256u; i += 64u) wm[i] = 0ull;
  uint64_t cyc[5] = {0ull, 0ull, 0ull, 0ull, 0ull};

  for (uint64_t t = blockIdx.x; t < p.trial_count; t += gridDim.x) {
    const uint64_t trial = p.trial_begin + t;
    const uint32_t tlo = (uint32_t)trial, thi = (uint32_t)(trial >> 32);
    const uint64_t t_start = stats ? __builtin_amdgcn_s_memtime() : 0ull;
    const uint64_t w_start = stats ? (uint64_t)wall_clock64() : 0ull;
    // ---- node.ts:21-26 (lane = node): faulty nodes killed with x = k = null
    const uint32_t myid = lane < m ? p.live_ids[lane] : 0xFFFFFFFFu;   // compact lane c -> node id
    uint64_t live = 0ull;
    for (uint32_t c = 0; c < m; ++c) live |= 1ull << rl(myid, c);
    uint64_t killed = all & ~live, decided = 0ull;
    uint32_t X = 0xFFFFFFFFu, K = 0xFFFFFFFFu, CI = 0u;
    for (uint32_t c = 0; c < m; ++c) CI = lane == rl(myid, c) ? c : CI;
    if ((live >> lane) & 1ull) {
      int32_t v;
      if (p.init_mode == BO_INIT_RANDOM) {        // oracle_random_init
        if (m <= 32u) {
          v = (int32_t)((init_word_small(k0, k1, trial) >> CI) & 1u);
        } else {
          const uint4 ir = philox4x32_10<false>(k0, k1, make_uint4(tlo, thi, CI >> 7, kStreamInit << 24));
          v = (int32_t)((coin_word_v(ir, ((CI >> 5) & 3u) + 1u) >> (CI & 31u)) & 1u);
        }
      } else {
        v = p.init_x[lane];
      }
      X = (uint32_t)v;
      K = 1u;                                      // /start: k = 1 (node.ts:172)
    }
    for (uint32_t s = lane; s < 128u; s += 64u) ibox[s] = s < 2u * N && ((live >> (s >> 1)) & 1ull) ? 0ull : kDead;
    if (lane < 4u) comp[lane] = 0ull;
    // ---- /start (node.ts:167-188): every live node broadcasts its x, in node order
    for (uint32_t c = 0; c < m; ++c) {
      const uint32_t body = ((rl(X, rl(myid, c)) & 3u) << 13) | (1u << 15);
      if (lane < N) pool[c * N + lane] = lane | body;
    }
    lds_order();
    uint64_t rng;
    {
      const uint4 o = philox4x32_10<false>(k0, k1, make_uint4(tlo, thi, 0u, kStreamOrder << 24));
      rng = (((uint64_t)o.x << 32) | o.y) ^ 0xD1B54A32D192ED03ull;
    }
    uint32_t next = 0;
    uint64_t next_key = uni64(p.ev_nstops ? p.ev_stops[0] : ~0ull);
    uint32_t len = m * N, cur = 1u, R = 0u, halted = 0u, overflow = 0u;
    uint64_t e = 0, batches = 0, trig = 0, c_z = stats ? __builtin_amdgcn_s_memtime() : 0ull;
    auto advance = [&]() {                         // node.ts:116-145 as DESIGN §2
      for (;;) {
        const uint64_t cw = uni64(comp[cur & 3u]);
        if ((cw | killed) != all) return;
        if ((decided | killed) == all) { halted = 1u; R = cur; return; }
        if (cur >= kmax) { halted = 2u; R = cur; return; }
        if (lane == 0u) comp[cur & 3u] = 0ull;
        lds_order();
        ++cur;
      }
    };
    auto kill = [&](uint32_t i) {                  // GET /stop (node.ts:191-194): drops every later message
      killed |= 1ull << i;
      if (lane < 2u && i < N) ibox[2u * i + lane] |= kDead;
      lds_order();
    };
    while (!halted) {
      // ---- scheduled GET /stop before delivery e
      bool crashed = false;
      while ((next_key >> 12) == e) {
        kill((uint32_t)(next_key & 4095u));
        crashed = true;
        ++next;
        next_key = uni64(next < p.ev_nstops ? p.ev_stops[next] : ~0ull);
      }
      if (box && poll_clock() - polled >= kPollCycles) {
        // live GET /stop requests (applied one poll after their sequence word,
        // so a burst lands together) and GET /getState snapshot requests
        const uint64_t req = apply_next ? uni64(pv_req) : 0ull;
        const uint32_t seq = rl(pv_word, 1u), sreq = rl(pv_word, 2u);
        apply_next = seq != seq_seen;
        seq_seen = seq;
        const uint64_t fresh = req & all & ~killed;
        for (uint64_t f = fresh; f; f &= f - 1ull) {
          const uint32_t i = (uint32_t)__builtin_ctzll(f);
          kill(i);
          if (lane == 0u)
            __hip_atomic_store(box + kLiveEv + i, e < 0xFFFFFFFFull ? (uint32_t)e : 0xFFFFFFFEu, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
        crashed = crashed || fresh != 0ull;
        if (crashed) {
          if (killed == all) { halted = 3u; break; }
          advance();
          if (halted) break;
          crashed = false;
        }
        if (sreq != snap_served) {
          // GET /getState (node.ts:197-199) mid-run: every node's state before delivery e
          snap_served = sreq;
          if (lane < N) {
            const bool f = (int32_t)K < 0 && (int32_t)X < 0;
            const uint32_t kl = (uint32_t)((killed >> lane) & 1ull) | ((X & 0xFFu) << 8) |
                                ((f ? 0xFFu : (uint32_t)((decided >> lane) & 1ull)) << 16);
            __hip_atomic_store(box + kSnapSt + 2u * lane, kl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(box + kSnapSt + 2u * lane + 1u, K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          if (lane == 0u) {
            __hip_atomic_store(box + kSnapE, (uint32_t)e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(box + kSnapE + 1u, (uint32_t)(e >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          __builtin_amdgcn_s_waitcnt(0x0F70);      // vmcnt(0): the states reached the host
          if (lane == 0u) __hip_atomic_store(box + kSnapSeq, sreq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        poll_issue();
      }
      if (crashed) {
        if (killed == all) { halted = 3u; break; }
        advance();
        if (halted) break;
      }
      if (len == 0u) { halted = 3u; break; }
      // ---- a micro-batch of events e .. e + B - 1 (lane i: event e + i)
      const uint64_t c_a = stats ? __builtin_amdgcn_s_memtime() : 0ull;
      uint32_t B = len < 64u ? len : 64u;
      if (next_key != ~0ull && (next_key >> 12) - e < B) B = (uint32_t)((next_key >> 12) - e);
      const bool act = lane < B;
      uint32_t qi = 0u, ti = 0u;
      bool wr = false;
      if (act) {
        const uint64_t z = smix(rng + (uint64_t)(lane + 1u) * kGm);
        qi = (uint32_t)(((uint64_t)(uint32_t)(z >> 32) * (uint64_t)(len - lane)) >> 32);
        ti = len - 1u - lane;
        wr = qi != ti;                             // event i moves the tail word t_i to q_i
        qarr[lane] = qi;
        if (wr) atomicOr(reinterpret_cast<unsigned long long *>(&wm[qi & 255u]), 1ull << lane);
      }
      lds_order();
      // the word at position pp before event ii: the word event j (the last
      // earlier writer of pp) moved there from t_j = len - 1 - j, before j;
      // pp never was a tail (pp < len - ii), so the chain ends in the pool
      auto word_at = [&](uint32_t pp, uint32_t ii) {
        for (;;) {
          uint64_t mm = wm[pp & 255u] & ((1ull << ii) - 1ull);
          uint32_t j = 64u;
          while (mm) {
            const uint32_t c = 63u - (uint32_t)__builtin_clzll(mm);
            if (qarr[c] == pp) { j = c; break; }
            mm &= ~(1ull << c);
          }
          if (j == 64u) return pool[pp];
          pp = len - 1u - j;
          ii = j;
        }
      };
      const uint32_t pv = act ? word_at(qi, lane) : 0u;
      const uint64_t c_b = stats ? __builtin_amdgcn_s_memtime() : 0ull;
      // ---- POST /message (node.ts:45-158): the batch's deliveries at once
      uint64_t inc = 0ull;
      uint32_t slot = 0u;
      if (act) {
        const uint32_t to = pv & 4095u, ph = (pv >> 12) & 1u, xv = (pv >> 13) & 3u;
        const uint32_t k = cur + (((pv >> 15) - cur) & 3u);
        slot = 2u * to + ph;
        if (k < kmax + 3u)                         // beyond the oracle's round window: dropped
          inc = (1ull << 26) + (xv == 0u ? 1ull : (xv == 1u ? 1ull << 13 : 0ull));
      }
      bool cross = false;
      if (inc) {
        const uint64_t old = __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(&ibox[slot]), inc,
                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        // killed receivers drop the message (node.ts:45): their slot counts
        // on, never tested; a live slot crosses its quorum (node.ts:52, :88)
        cross = !(old & kDead) && ((old >> 26) & kF13) + 1u == quorum;
      }
      uint32_t tr = 0xFFFFFFFFu;
      for (uint64_t xm = __ballot(cross); xm; xm &= xm - 1ull) {
        // a crossed slot triggers at the last batch event into it
        const uint32_t s = rl(slot, (uint32_t)__builtin_ctzll(xm));
        const uint64_t into = __ballot(inc != 0ull && slot == s);
        const uint32_t last = 63u - (uint32_t)__builtin_clzll(into);
        tr = last < tr ? last : tr;
      }
      uint32_t used = B;
      if (tr != 0xFFFFFFFFu) {
        if (inc && lane > tr)                      // the batch ends at its first trigger: later adds undone
          __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(&ibox[slot]), 0ull - inc, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        used = tr + 1u;
      }
      const uint64_t c_c = stats ? __builtin_amdgcn_s_memtime() : 0ull;
      // ---- the pool after the batch: each position below the new length that
      // the batch wrote keeps its last writer's word
      bool last = false;
      if (lane < used && wr && qi < len - used) {
        const uint64_t below = used >= 64u ? ~0ull : (1ull << used) - 1ull;
        uint64_t mm = wm[qi & 255u] & below & ~((2ull << lane) - 1ull);
        last = true;
        while (mm) {
          const uint32_t c = (uint32_t)__builtin_ctzll(mm);
          if (qarr[c] == qi) { last = false; break; }
          mm &= mm - 1ull;
        }
      }
      const uint32_t wv = last ? word_at(ti, lane) : 0u;
      lds_order();
      if (last) pool[qi] = wv;
      if (wr) wm[qi & 255u] = 0ull;
      lds_order();
      len -= used;
      e += used;
      rng += (uint64_t)used * kGm;
      ++batches;
      if (stats) {
        const uint64_t c_d = __builtin_amdgcn_s_memtime();
        cyc[0] += c_a - c_z;
        cyc[1] += c_b - c_a;
        cyc[2] += c_c - c_b;
        cyc[3] += c_d - c_c;
        c_z = c_d;
      }
      if (tr == 0xFFFFFFFFu) continue;
      // ---- the trigger (node.ts:52-80 R-phase, :88-157 P-phase)
      const uint32_t msg = rl(pv, tr), ts = rl(slot, tr);
      const uint32_t to = msg & 4095u, ph = (msg >> 12) & 1u;
      const uint32_t k = cur + (((msg >> 15) - cur) & 3u);
      const uint64_t v = uni64(ibox[ts]);
      if (lane == 0u) ibox[ts] = 0ull;             // every message of the phase arrived: the slot is free
      lds_order();
      const uint32_t c0 = (uint32_t)(v & kF13), c1 = (uint32_t)((v >> 13) & kF13);
      uint32_t body = 0xFFFFFFFFu;
      if (ph == 0u) {
        const uint32_t pr = c0 > c1 ? 0u : (c1 > c0 ? 1u : 2u);
        body = (1u << 12) | (pr << 13) | ((k & 3u) << 15);
      } else {
        uint32_t nx;
        bool dec = true;
        if (c0 > F) nx = 0u;
        else if (c1 > F) nx = 1u;
        else {
          dec = false;
          if (c0 + c1 > 0u && c0 > c1) nx = 0u;
          else if (c0 + c1 > 0u && c0 < c1) nx = 1u;
          else {
            const uint32_t c = rl(CI, to);         // the coin of compact node c in round k (node.ts:111)
            const uint4 rr = coin_block<false>(k0, k1, tlo, thi, c, k);
            nx = uni((coin_word(rr, k) >> (c & 31u)) & 1u);
          }
        }
        X = wl(X, nx, to);
        K = wl(K, k + 1u, to);
        if (dec) decided |= 1ull << to;
        if (lane == 0u) comp[k & 3u] |= 1ull << to;
        lds_order();
        advance();
        if (!halted) body = (nx << 13) | (((k + 1u) & 3u) << 15);
      }
      if (body != 0xFFFFFFFFu) {                   // the broadcast to all N nodes
        if (len + N > cap) {
          overflow = 1u;
          halted = 3u;
          break;
        }
        if (lane < N) pool[len + lane] = lane | body;
        len += N;
        lds_order();
      }
      ++trig;
      if (stats) {
        const uint64_t c_d = __builtin_amdgcn_s_memtime();
        cyc[4] += c_d - c_z;
        c_z = c_d;
      }
    }
    // ---- outcome over the nodes still running
    const bool run = lane < N && !((killed >> lane) & 1ull);
    const bool g0 = __any(run && X == 0u), g1 = __any(run && X == 1u), gq = __any(run && X != 0u && X != 1u);
    const bool gl = __any(run);
    const uint32_t vv = (!gl || gq || (g0 && g1)) ? 2u : (g1 ? 1u : 0u);
    if (lane == 0u) {
      atomicAdd(&p.hist[halted == 1u ? (R * 3u + vv) : vv], 1ull);
      if (halted == 1u && vv == 2u) atomicAdd(&p.hist[p.hist_len - 1u], 1ull);
      if (overflow && p.rounds_out) atomicOr(p.rounds_out, 0x80000000u);
      if (overflow && p.overflow) atomicOr(p.overflow, 2u);
      if (p.node_out && p.rounds_out) atomicOr(p.rounds_out, halted == 1u ? R : 0u);
      if (stats) {
        atomicAdd(&stats[0], (unsigned long long)batches);
        atomicAdd(&stats[1], (unsigned long long)e);
        atomicAdd(&stats[3], (unsigned long long)trig);
        atomicAdd(&stats[5], (unsigned long long)cyc[0]);
        atomicAdd(&stats[6], (unsigned long long)cyc[1]);
        atomicAdd(&stats[8], (unsigned long long)cyc[2]);
        atomicAdd(&stats[10], (unsigned long long)cyc[3]);
        atomicAdd(&stats[11], (unsigned long long)cyc[4]);
        atomicAdd(&stats[12], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start));
        atomicAdd(&stats[13], (unsigned long long)((uint64_t)wall_clock64() - w_start));
      }
    }
    if (p.node_out && lane < N) {
      bo_node_state ns;
      const bool f = (int32_t)K < 0 && (int32_t)X < 0;   // faulty from launch (never ran)
      ns.killed = (int8_t)((killed >> lane) & 1ull);
      ns.x = (int8_t)X;
      ns.decided = f ? (int8_t)-1 : (int8_t)((decided >> lane) & 1ull);
      ns.pad = 0;
      ns.k = (int32_t)K;
      p.node_out[lane] = ns;
    }
    lds_order();
  }
  if (box) __builtin_amdgcn_s_waitcnt(0x0F70);     // the last poll lands before the wave ends
}

// ---------------------------------------------------------------------------
// The smallest networks (N <= kEventRegMaxN): one wave, one event per step,
// no memory.  At N = 10 a batch of the wave kernel above carries ~10 events
// (it ends at its first trigger, and every ~10th delivery is one) for ~730
// instructions and ~30 LDS round trips (tools/live_profile.py, PMC).  Here
// the whole round state lives in registers:
//   * the pool in R VGPRs, position p in lane p & 63 of register p >> 6
//     (R * 64 >= 4N^2 + 64); a step reads its two words with v_readlane
//     through a uniform register index (s_set_gpr_idx) and writes the moved
//     word back with one lane select -- about 15 instructions, no waits;
//   * the inbox slots in one VGPR, slot s = 2 * to + ph in lane s, packed
//     {len << 24 | c1 << 16 | c0 << 8}: a pool word carries its slot, k & 3
//     and the increment its delivery adds, so a delivery is one read-add-select;
//   * 64 picks per block (lane i: the pick word of event e + i, splitmix64
//     is a counter), one readlane per event;
//   * while the pool holds <= 64 words (at N = 10, F = 5 it never holds more
//     than ~50) it lives in one VGPR alone, and the array form starts at the
//     first broadcast past 64 (no register-array copies around a trigger);
//   * the trigger, the stops, the mailbox and the snapshots as the wave
//     kernel, node state in lane registers and 32-bit SGPR masks, the four
//     open rounds' completion masks packed in one 64-bit scalar.
// Words: slot | (k & 3) << 6 | {1 << 24 | (x == 0) << 8 | (x == 1) << 16}.
// At N = 10, F = 5 a batch (~10 deliveries and a trigger) takes ~3050 shader
// cycles (r06-F: 3600): ~2070 the deliveries (~207 each: three v_readlane ->
// SALU hops), ~1000 the loop head and the trigger (~330 / ~720 with phase
// stamps in r06-G5, since dropped: their SGPRs cost 6 %).  A/Bs of each change
// on one box: profiles/r06-G_reg_kernel_ab.jsonl (register allocation moves
// these numbers by several % either way, e.g. dropping the one remaining
// cycle stamp costs 2-14 %: keep changes here under an A/B).
template <int R, bool SM>
__global__ void __launch_bounds__(64) benor_event_reg_kernel(KParams p) {
  using M = uint32_t;                                                 // node masks (N <= 16)
  const uint32_t lane = threadIdx.x;
  const uint32_t N = p.N, F = p.F, quorum = p.N - p.F, m = p.m, kmax = p.k_max, cap = p.ev_cap;
  const M all = (M(1) << N) - M(1);                                   // N <= kEventRegMaxN
  const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
  uint32_t *box = p.live_box;
  unsigned long long *const stats = p.ev_stats;
  // the request word's low half (N <= 16): a 64-bit load whose high half is
  // dead lets the register allocator reuse that half, and the reuse waits for
  // the host-memory load at the next batch end
  uint32_t pv_req = 0u;
  uint32_t pv_word = 0u, snap_served = 0u, seq_seen = 0u;
  bool apply_next = false;
  long long polled = 0;
  auto poll_issue = [&]() {
    if (lane == 0u) pv_req = __hip_atomic_load(box + kLiveReq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 1u) pv_word = __hip_atomic_load(box, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 2u) pv_word = __hip_atomic_load(box + kSnapReq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    polled = poll_clock();
  };
  if (box) poll_issue();
  auto rl = [](uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); };
  auto wl = [lane](uint32_t v, uint32_t val, uint32_t l) { return lane == l ? val : v; };   // lane l of v := val
  auto inc_of = [](uint32_t x) { return (1u << 24) | (x == 0u ? 1u << 8 : (x == 1u ? 1u << 16 : 0u)); };
  uint32_t P[R];

  for (uint64_t t = blockIdx.x; t < p.trial_count; t += gridDim.x) {
    const uint64_t trial = p.trial_begin + t;
    const uint32_t tlo = (uint32_t)trial, thi = (uint32_t)(trial >> 32);
    uint64_t t_start = stats ? __builtin_amdgcn_s_memtime() : 0ull;
    uint64_t w_start = stats ? (uint64_t)wall_clock64() : 0ull;
    asm volatile("" : "+v"(t_start), "+v"(w_start));   // cold: kept out of the SGPR file
    // ---- node.ts:21-26 (lane = node): faulty nodes killed with x = k = null
    const uint32_t myid = lane < m ? p.live_ids[lane] : 0xFFFFFFFFu;   // compact lane c -> node id
    M live = 0;
    for (uint32_t c = 0; c < m; ++c) live |= M(1) << rl(myid, c);
    M killed = all & ~live, decided = 0;
    uint32_t X = 0xFFFFFFFFu, K = 0xFFFFFFFFu, CI = 0u;
    for (uint32_t c = 0; c < m; ++c) CI = lane == rl(myid, c) ? c : CI;
    if (lane < N && ((live >> lane) & 1u)) {
      int32_t v;
      if (p.init_mode == BO_INIT_RANDOM) {        // oracle_random_init (m <= 32)
        v = (int32_t)((init_word_small(k0, k1, trial) >> CI) & 1u);
      } else {
        v = p.init_x[lane];
      }
      X = (uint32_t)v;
      K = 1u;                                      // /start: k = 1 (node.ts:172)
    }
    // ---- /start (node.ts:167-188): every live node broadcasts its x, in node order
    const uint32_t XC = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(myid << 2), (int)X);   // x of compact node c
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t pos = (uint32_t)r * 64u + lane, c = pos / N, n = pos - c * N;
      const uint32_t xc = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(c << 2), (int)XC);
      P[r] = c < m ? (2u * n) | (1u << 6) | inc_of(xc & 3u) : 0u;
    }
    // inbox slots; bit 7: the receiver is killed
    uint32_t CNT = lane < 2u * N && !((live >> (lane >> 1)) & 1u) ? 0x80u : 0u;
    // round k complete: the nodes done with it in bits 16 (k & 3) .. + 15 of one scalar
    uint64_t CPV = 0ull;
    auto comp_get = [&](uint32_t i) -> M { return (M)((CPV >> (16u * i)) & 0xFFFFull); };
    auto comp_set = [&](uint32_t i, M v) { CPV = (CPV & ~(0xFFFFull << (16u * i))) | ((uint64_t)v << (16u * i)); };
    uint64_t rngb;
    {
      const uint4 o = philox4x32_10<false>(k0, k1, make_uint4(tlo, thi, 0u, kStreamOrder << 24));
      rngb = (((uint64_t)o.x << 32) | o.y) ^ 0xD1B54A32D192ED03ull;
    }
    uint32_t next = 0;
    uint64_t next_key = uni64(p.ev_nstops ? p.ev_stops[0] : ~0ull);
    uint64_t next_e = next_key >> 12;              // the next scheduled stop's delivery (2^52 - 1: none)
    uint32_t len = m * N, cur = 1u, Rr = 0u, halted = 0u, overflow = 0u;
    uint64_t e = 0, trig = 0, cyc_steps = 0;
    uint32_t H = 0u, hi = 64u;                     // the block's picks, the next one's lane
    auto advance = [&]() {                         // node.ts:116-145 as DESIGN §2
      for (;;) {
        const M cw = comp_get(cur & 3u);
        if ((cw | killed) != all) return;
        if ((decided | killed) == all) { halted = 1u; Rr = cur; return; }
        if (cur >= kmax) { halted = 2u; Rr = cur; return; }
        comp_set(cur & 3u, 0);
        ++cur;
      }
    };
    auto kill = [&](uint32_t i) {                  // GET /stop (node.ts:191-194): drops every later message
      killed |= M(1) << i;
      CNT |= (lane >> 1) == i ? 0x80u : 0u;
    };
    auto pread = [&](uint32_t pos) { return rl(P[pos >> 6], pos & 63u); };
    // While the pool fits one register (len <= 64; at N = 10, F = 5 it
    // never holds more than ~50 words) it lives in P0 alone and the array P
    // is untouched; the batch that outgrows P0 writes it back to P[0] and
    // the run goes on in the array form.  One batch: 0 go on, 1 the run
    // ended, 2 the pool left P0.
    uint32_t P0 = P[0];
    auto batch = [&](auto small) -> uint32_t {
      // ---- scheduled GET /stop before delivery e
      bool crashed = false;
      while (next_e == e) {
        kill((uint32_t)(next_key & 4095u));
        crashed = true;
        ++next;
        next_key = uni64(next < p.ev_nstops ? p.ev_stops[next] : ~0ull);
        next_e = next_key >> 12;
      }
      if (box && hi == 64u) {                      // the clock is read once per 64 events
        if (poll_clock() - polled >= kPollCycles) {
          // live GET /stop requests (applied one poll after their sequence
          // word) and GET /getState snapshot requests, as the wave kernel
          const uint32_t req = apply_next ? uni(pv_req) : 0u;
          const uint32_t seq = rl(pv_word, 1u), sreq = rl(pv_word, 2u);
          apply_next = seq != seq_seen;
          seq_seen = seq;
          const M fresh = (M)req & all & ~killed;
          for (M f = fresh; f; f &= f - 1) {
            const uint32_t i = (uint32_t)__builtin_ctzll((uint64_t)f);
            kill(i);
            if (lane == 0u)
              __hip_atomic_store(box + kLiveEv + i, e < 0xFFFFFFFFull ? (uint32_t)e : 0xFFFFFFFEu, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
          }
          crashed = crashed || fresh != 0ull;
          if (sreq != snap_served) {
            // GET /getState (node.ts:197-199) mid-run: every node's state before delivery e
            snap_served = sreq;
            if (lane < N) {
              const bool f = (int32_t)K < 0 && (int32_t)X < 0;
              const uint32_t kl = (uint32_t)((killed >> lane) & 1u) | ((X & 0xFFu) << 8) |
                                  ((f ? 0xFFu : (uint32_t)((decided >> lane) & 1u)) << 16);
              __hip_atomic_store(box + kSnapSt + 2u * lane, kl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              __hip_atomic_store(box + kSnapSt + 2u * lane + 1u, K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (lane == 0u) {
              __hip_atomic_store(box + kSnapE, (uint32_t)e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              __hip_atomic_store(box + kSnapE + 1u, (uint32_t)(e >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);    // vmcnt(0): the states reached the host
            if (lane == 0u) __hip_atomic_store(box + kSnapSeq, sreq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          poll_issue();
        }
      }
      if (crashed) {
        if (killed == all) { halted = 3u; return 1u; }
        advance();
        if (halted) return 1u;
      }
      if (len == 0u) { halted = 3u; return 1u; }
      if (hi == 64u) {                             // the next 64 picks (event e + i in lane i)
        const uint64_t z = smix(rngb + (uint64_t)(lane + 1u) * kGm);
        H = (uint32_t)(z >> 32);
        rngb += 64ull * kGm;
        hi = 0u;
      }
      // ---- POST /message (node.ts:45-158), one delivery per step up to the
      // block's end, the next stop or the first trigger
      uint32_t seg = 64u - hi;
      if (seg > len) seg = len;
      if (next_e - e < seg) seg = (uint32_t)(next_e - e);   // e < next_e here
      uint32_t j = 0u, tw = 0u, tc = 0u;
      bool fired = false;
      seg = uni(seg);
      const uint32_t qmark = quorum << 24;
      // one delivery: false when its slot reaches the quorum (the trigger)
      auto deliver = [&](uint32_t w, auto late) {  // late: messages of round >= k_max + 3 are dropped
        if (decltype(late)::value && cur + (((w >> 6) - cur) & 3u) >= kmax + 3u) return true;
        // one register: the slot through the SALU (a v_readlane lane select
        // written by the previous v_readlane stalls longer; r06-G5, 4 % per
        // event at N = 10; in the array form it costs, r06-G7)
        uint32_t s = w & 63u;
        if constexpr (decltype(small)::value) asm volatile("s_and_b32 %0, %1, 63" : "=s"(s) : "s"(w));
        const uint32_t c = rl(CNT, s) + (w & 0xFFFFFF00u);
        CNT = wl(CNT, c, s);
        // killed receivers drop the message (node.ts:45): their slots count
        // on (wrapping), never tested; a live slot reaches its quorum
        if ((c & 0xFF000080u) != qmark) return true;
        tw = w;
        tc = c;
        fired = true;
        return false;
      };
      auto steps = [&](auto late) {
        if constexpr (decltype(small)::value && !decltype(late)::value) {
          // the common case, one register and no late drops: one exit test
          // per delivery (the segment's end or a quorum)
          uint32_t Q0 = P0, rem = seg, w = 0u, c = 0u;
          if (rem) {
            for (;;) {
              len = uni(len);
              const uint32_t q = uni((uint32_t)(((uint64_t)rl(H, hi + j) * len) >> 32));
              w = rl(Q0, q);
              --len;
              const uint32_t tv = rl(Q0, len);
              Q0 = lane == q ? tv : Q0;            // the tail word moves to q
              ++j;
              --rem;
              uint32_t s;
              asm volatile("s_and_b32 %0, %1, 63" : "=s"(s) : "s"(w));
              c = rl(CNT, s) + (w & 0xFFFFFF00u);
              CNT = wl(CNT, c, s);
              const uint32_t x = (c & 0xFF000080u) ^ qmark;   // 0: a live slot reached its quorum
              if (uni(x < rem ? x : rem) == 0u) break;
            }
            if ((c & 0xFF000080u) == qmark) {
              tw = w;
              tc = c;
              fired = true;
            }
          }
          P0 = Q0;
          return;
        }
        if (decltype(small)::value || len <= 64u) {   // the whole pool in lane p of one register
          uint32_t Q0 = decltype(small)::value ? P0 : P[0];
          while (j < seg) {
            j = uni(j);
            len = uni(len);
            const uint32_t q = uni((uint32_t)(((uint64_t)rl(H, hi + j) * len) >> 32));
            const uint32_t w = rl(Q0, q);
            --len;
            const uint32_t tv = rl(Q0, len);
            Q0 = lane == q ? tv : Q0;              // the tail word moves to q
            ++j;
            if (!deliver(w, late)) break;
          }
          if (decltype(small)::value) P0 = Q0;
          else P[0] = Q0;
          return;
        }
        while (j < seg) {
          j = uni(j);
          len = uni(len);
          const uint32_t q = uni((uint32_t)(((uint64_t)rl(H, hi + j) * len) >> 32));
          const uint32_t w = pread(q);
          --len;
          {                                        // the tail word moves to q (no-op when q is the tail)
            const uint32_t tv = pread(len);
            uint32_t reg = P[q >> 6];
            reg = wl(reg, tv, q & 63u);
            P[q >> 6] = reg;
          }
          ++j;
          if (!deliver(w, late)) break;
        }
      };
      const uint64_t c_a = stats ? __builtin_amdgcn_s_memtime() : 0ull;
      if (cur >= kmax) steps(std::true_type{});
      else steps(std::false_type{});
      if (stats) cyc_steps += __builtin_amdgcn_s_memtime() - c_a;
      e += j;
      hi += j;
      if (!fired) return 0u;
      ++trig;
      // ---- the trigger (node.ts:52-80 R-phase, :88-157 P-phase)
      const uint32_t s = tw & 63u, to = s >> 1, ph = s & 1u;
      const uint32_t k = cur + (((tw >> 6) - cur) & 3u);
      CNT = wl(CNT, 0u, s);                        // every message of the phase arrived: the slot is free
      const uint32_t c0 = (tc >> 8) & 0xFFu, c1 = (tc >> 16) & 0xFFu;
      uint32_t base = 0xFFFFFFFFu;
      if (ph == 0u) {
        const uint32_t pr = c0 > c1 ? 0u : (c1 > c0 ? 1u : 2u);
        base = 1u | ((k & 3u) << 6) | inc_of(pr);
      } else {
        uint32_t nx;
        bool dec = true;
        if (c0 > F) nx = 0u;
        else if (c1 > F) nx = 1u;
        else {
          dec = false;
          if (c0 + c1 > 0u && c0 > c1) nx = 0u;
          else if (c0 + c1 > 0u && c0 < c1) nx = 1u;
          else {
            const uint32_t c = rl(CI, to);         // the coin of compact node c in round k (node.ts:111)
            const uint4 rr = coin_block<false>(k0, k1, tlo, thi, c, k);
            nx = uni((coin_word(rr, k) >> (c & 31u)) & 1u);
          }
        }
        X = wl(X, nx, to);
        K = wl(K, k + 1u, to);
        if (dec) decided |= M(1) << to;
        comp_set(k & 3u, comp_get(k & 3u) | (M(1) << to));
        advance();
        if (!halted) base = ((((k + 1u) & 3u) << 6)) | inc_of(nx);
      }
      if (base != 0xFFFFFFFFu) {                   // the broadcast to all N nodes: positions len .. len + N - 1
        if (decltype(small)::value && len + N <= 64u) {   // (cap >= 4 N^2 + 64 > 64)
          const uint32_t d = lane - len;
          P0 = d < N ? 2u * d + base : P0;
          len += N;
          return 0u;
        }
        if (len + N > cap) {
          overflow = 1u;
          halted = 3u;
          return 1u;
        }
        if (decltype(small)::value) P[0] = P0;     // the pool outgrows one register
        const uint32_t r0 = len >> 6, r1 = (len + N - 1u) >> 6;
        if (r1 == 0u) {                            // within register 0
          const uint32_t d = lane - len;
          P[0] = d < N ? 2u * d + base : P[0];
        } else {
          const uint32_t d = r0 * 64u + lane - len;
          uint32_t reg = P[r0];
          reg = d < N ? 2u * d + base : reg;
          P[r0] = reg;
        }
        if (r1 != r0) {
          const uint32_t d = r1 * 64u + lane - len;
          uint32_t reg = P[r1];
          reg = d < N ? 2u * d + base : reg;
          P[r1] = reg;
        }
        len += N;
        if (decltype(small)::value) return 2u;
      }
      return 0u;
    };
    if constexpr (SM) {                            // SM: the launch's pool starts in one register
      bool grown = len > 64u;
      while (!halted && !grown) {
        const uint32_t r = batch(std::true_type{});
        if (r == 1u) break;
        grown = r == 2u;
      }
    }
    while (!halted) {
      if (batch(std::false_type{}) == 1u) break;
    }
    // ---- outcome over the nodes still running
    const bool run = lane < N && !((killed >> lane) & 1u);
    const bool g0 = __any(run && X == 0u), g1 = __any(run && X == 1u), gq = __any(run && X != 0u && X != 1u);
    const bool gl = __any(run);
    const uint32_t vv = (!gl || gq || (g0 && g1)) ? 2u : (g1 ? 1u : 0u);
    if (lane == 0u) {
      atomicAdd(&p.hist[halted == 1u ? (Rr * 3u + vv) : vv], 1ull);
      if (halted == 1u && vv == 2u) atomicAdd(&p.hist[p.hist_len - 1u], 1ull);
      if (overflow && p.rounds_out) atomicOr(p.rounds_out, 0x80000000u);
      if (overflow && p.overflow) atomicOr(p.overflow, 2u);
      if (p.node_out && p.rounds_out) atomicOr(p.rounds_out, halted == 1u ? Rr : 0u);
      if (stats) {
        atomicAdd(&stats[0], (unsigned long long)trig);
        atomicAdd(&stats[1], (unsigned long long)e);
        atomicAdd(&stats[3], (unsigned long long)trig);
        atomicAdd(&stats[6], (unsigned long long)cyc_steps);
        atomicAdd(&stats[12], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start));
        atomicAdd(&stats[13], (unsigned long long)((uint64_t)wall_clock64() - w_start));
      }
    }
    if (p.node_out && lane < N) {
      bo_node_state ns;
      const bool f = (int32_t)K < 0 && (int32_t)X < 0;   // faulty from launch (never ran)
      ns.killed = (int8_t)((killed >> lane) & 1u);
      ns.x = (int8_t)X;
      ns.decided = f ? (int8_t)-1 : (int8_t)((decided >> lane) & 1u);
      ns.pad = 0;
      ns.k = (int32_t)K;
      p.node_out[lane] = ns;
    }
  }
  if (box) __builtin_amdgcn_s_waitcnt(0x0F70);     // the last poll lands before the wave ends
}

uint32_t event_wg_waves(const KParams &p) {
  const uint32_t forced = knob_u32("BENOR_LIVE_WAVES", 0u);
  if (forced == 1u || forced == 3u || forced == 7u || forced == 15u) return forced;
  if (p.N <= 32u) return 1u;
  if (p.N <= 128u) return 3u;
  if (p.N <= 512u) return 7u;
  return 15u;
}

bool event_wg_lds_pool(const KParams &p) { return (uint64_t)p.ev_cap * 4u <= kEventBigLdsPool; }

static uint32_t wg_lds_bytes(const KParams &p, uint32_t W, uint32_t HS) {
  const uint32_t N = p.N;
  uint32_t b = ((uint32_t)sizeof(Ctl) + 15u) & ~15u;
  b += 16u * N + 8u * 64u * 6u + 8u * HS + 8u * 64u + 8u * p.ev_rstops;   // ibox, killed/decided/comp, hash, Floyd set, keys
  b += 8u * N + 3u * 4u * 64u * W;                                        // smax; bmax, nxt, tvs
  b += 2u * ((N + 7u) & ~7u) * 2u + ((N + 15u) & ~15u);                   // ks, cidx, xs
  if (event_wg_lds_pool(p)) b += 4u * p.ev_cap;
  return b;
}

uint32_t event_wg_hash_slots(const KParams &p, uint32_t W) {
  for (uint32_t f = 8u; f > 2u; f >>= 1) {
    const uint32_t hs = pow2_ceil(f * 64u * W);
    if (wg_lds_bytes(p, W, hs) <= 150u * 1024u) return hs;
  }
  return pow2_ceil(2u * 64u * W);
}

uint32_t event_wg_lds_bytes(const KParams &p, uint32_t W) { return wg_lds_bytes(p, W, event_wg_hash_slots(p, W)); }

template <int W, bool LP, bool ST>
static hipError_t launch_wg1(KParams p, int grid, hipStream_t s) {
  p.ev_hs = event_wg_hash_slots(p, (uint32_t)W);
  const uint32_t lds = event_wg_lds_bytes(p, (uint32_t)W);
  if (lds > 64u * 1024u) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&benor_event_wg_kernel<W, LP, ST>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((benor_event_wg_kernel<W, LP, ST>), dim3(grid), dim3(64 * (W + 1)), lds, s, p);
  return hipGetLastError();
}

// the stamps and counters only where BENOR_EVENT_STATS asks for them: their
// registers slow the control wave otherwise
template <int W, bool LP>
static hipError_t launch_wg(KParams p, int grid, hipStream_t s) {
  return p.ev_stats ? launch_wg1<W, LP, true>(p, grid, s) : launch_wg1<W, LP, false>(p, grid, s);
}

// Small networks run on a one-wave kernel, unless a random /stop schedule
// (drawn by the workgroup kernel's control wave) or a forced wave count asks
// for the workgroup kernel.
static bool event_one_wave(const KParams &p) {
  return p.ev_rstops == 0u && knob_u32("BENOR_LIVE_WAVES", 0u) == 0u;
}

uint32_t event_reg_regs(const KParams &p) {
  if (p.N > kEventRegMaxN || !event_one_wave(p) || knob_is("BENOR_EVENT_FORM", "wave")) return 0u;
  const uint32_t need = (p.ev_cap + 63u) / 64u;
  return need <= 16u ? 16u : (need <= 32u ? 32u : 0u);
}

bool event_wave_form(const KParams &p) { return p.N <= kEventWaveMaxN && event_one_wave(p) && !event_reg_regs(p); }

uint32_t event_wave_lds_bytes(const KParams &p) {
  return 4u * ((p.ev_cap + 1u) & ~1u) + 4u * 64u + 8u * 256u + 8u * 128u + 8u * 4u;
}

hipError_t launch_event_wg(const KParams &p, int grid, hipStream_t s) {
  if (const uint32_t regs = event_reg_regs(p)) {
    // the one-register pool mode only where the pool starts there (m N <= 64):
    // compiled in, it slows the array form by 5-8 % (r06-G9, N = 12 and 16)
    const bool sm = p.m * p.N <= 64u;
    if (regs == 16u && sm) hipLaunchKernelGGL((benor_event_reg_kernel<16, true>), dim3(grid), dim3(64), 0, s, p);
    else if (regs == 16u) hipLaunchKernelGGL((benor_event_reg_kernel<16, false>), dim3(grid), dim3(64), 0, s, p);
    else if (sm) hipLaunchKernelGGL((benor_event_reg_kernel<32, true>), dim3(grid), dim3(64), 0, s, p);
    else hipLaunchKernelGGL((benor_event_reg_kernel<32, false>), dim3(grid), dim3(64), 0, s, p);
    return hipGetLastError();
  }
  if (event_wave_form(p)) {
    const uint32_t lds = event_wave_lds_bytes(p);
    const void *fn = p.ev_stats ? reinterpret_cast<const void *>(&benor_event_wave_kernel<true>)
                                : reinterpret_cast<const void *>(&benor_event_wave_kernel<false>);
    if (lds > 64u * 1024u) {
      const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    if (p.ev_stats) hipLaunchKernelGGL((benor_event_wave_kernel<true>), dim3(grid), dim3(64), lds, s, p);
    else hipLaunchKernelGGL((benor_event_wave_kernel<false>), dim3(grid), dim3(64), lds, s, p);
    return hipGetLastError();
  }
  const uint32_t W = event_wg_waves(p);
  const bool lp = event_wg_lds_pool(p);
  if (W == 1u) return lp ? launch_wg<1, true>(p, grid, s) : launch_wg<1, false>(p, grid, s);
  if (W == 3u) return lp ? launch_wg<3, true>(p, grid, s) : launch_wg<3, false>(p, grid, s);
  if (W == 7u) return lp ? launch_wg<7, true>(p, grid, s) : launch_wg<7, false>(p, grid, s);
  return lp ? launch_wg<15, true>(p, grid, s) : launch_wg<15, false>(p, grid, s);
}

}  // namespace benor
