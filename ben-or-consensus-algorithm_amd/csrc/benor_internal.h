// benor_internal.h -- launch-side contract between the C-ABI runtime
// (benor_runtime.cpp) and the gfx950 kernels (benor_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "benor.h"

namespace benor {

// Philox counter-stream tags (top byte of counter word 3).  Must match
// oracle/benor_oracle.c (the checker) -- DESIGN.md §3.
constexpr uint32_t kStreamCoin = 0u;
constexpr uint32_t kStreamInit = 1u;
constexpr uint32_t kStreamDelivery = 2u;
constexpr uint32_t kStreamOrder = 3u;
constexpr uint32_t kStreamCrash = 4u;

constexpr int kWavesPerBlock = 4;          // 256-thread workgroups, one trial per wave

constexpr uint32_t kMaxW = BO_MAX_N / 64;  // u64 words per bit plane at N = 4096
constexpr int kMaxWSpecialised = 32;       // m <= 2048: fully unrolled W-specialised kernel
constexpr uint32_t kMaxLaneM = 64;         // m <= 64: lane kernel, one trial per lane (benor_lane.h)
constexpr uint32_t kMaxSmallMfmaM = 32;    // 2 <= m <= 32: packed matrix-core kernel, 64 * min(32 / m, 8)
                                           // trials per wave iteration (benor_mfma_small.h)
constexpr uint32_t kMaxMfmaM = 1024;       // matrix-core kernel (benor_mfma.h): W <= 16, operands in registers;
                                           // beyond, the big-network form (runtime W, proposals in LDS) to BO_MAX_N
constexpr uint32_t kMaxEventN = 256;       // event level, one lane per trial: node ids in 8 bits of a message;
                                           // up to BO_MAX_N: one wave per trial (benor_event_big.hip)
// Workgroups of `lds` dynamic LDS bytes that fit one CU's 160 KB: allocation
// is in 512-byte granules (a 23216-byte group fits 6 per CU, not 7: the 7th
// waits, and a grid sized for 7 per CU ran 1.45x longer).
constexpr uint32_t lds_groups_per_cu(uint32_t lds) { return lds ? (160u * 1024u) / ((lds + 511u) & ~511u) : 64u; }
constexpr uint32_t kMaxEventLdsN = 31;     // event level: inbox counters in LDS (5-bit fields) up to here
constexpr uint64_t kMaxTrialsPerLaunch = 1ull << 31;   // trial offsets within a launch fit 32 bits
constexpr uint32_t kParamBytes = 32;       // LDS parameter block after the histogram (W kernel)

struct KParams {
  uint32_t N, F;            // network size, fault parameter
  uint32_t m;               // live (non-crashed) nodes = senders = receivers
  uint32_t W;               // u64 words per plane = ceil(m / 64) = receiver groups
  uint32_t G;               // receiver groups per tally block (template parameter); lane and matrix-core kernels: KIND
  uint32_t nblocks;         // ceil(W / G)
  uint32_t variant;         // 7: matrix-core lockstep, round 1 (benor_mfma.h; the W kernel serves its state
                            //    launches and the trials it defers),
                            // 8: packed matrix-core lockstep (2 <= m <= 32, benor_mfma_small.h; the lane kernel
                            //    serves its state launches),
                            // 6: lane lockstep (m <= 64), 1: W-specialised lockstep (W <= kMaxWSpecialised = 32),
                            // 0: blocked lockstep, 2: random delivery, 4: event level
  uint32_t base_variant;    // variant 7: the popcount kernel (1 W, 0 blocked) that serves the state
  uint32_t base_G;          //   launches and the deferred trials, and its G
  uint32_t mode;            // BO_MODE_LOCKSTEP / BO_MODE_RANDOM_DELIVERY
  uint32_t q;               // quorum N - F (messages each receiver tallies per phase)
  uint32_t k_max;
  uint32_t init_mode;       // BO_INIT_RANDOM / BO_INIT_FIXED
  uint32_t init_q;          // live nodes whose fixed initial value is "?" (0 for random init)
  uint32_t init_tie;        // fixed init: as many live 0s as 1s (every trial ties in round 1)
  uint32_t hist_len;        // (k_max + 1) * 3 + 1
  uint32_t lds_bytes;       // dynamic LDS per workgroup
  uint32_t wave_bytes;      // per-wave LDS region
  uint32_t hist_bytes;      // LDS histogram bytes (16-aligned)
  uint64_t seed;
  uint64_t trial_begin;
  uint64_t trial_count;
  const uint32_t *live_ids;        // [m] compact index -> node id (device)
  const uint4 *init_plane;         // [W] {X0lo, X0hi, X1lo, X1hi} (device; fixed init)
  unsigned long long *hist;        // [hist_len] (device, accumulated)
  bo_node_state *node_out;         // [N] (device) or nullptr; only with trial_count == 1
  uint32_t *rounds_out;            // (device) or nullptr
  // event-level mode (variant 4), N <= kMaxEventN
  uint64_t faulty_mask[4];         // node-id bitset, N <= 256
  const int8_t *init_x;            // [N] (device; fixed init)
  const uint32_t *crash_at;        // [N] (device) or nullptr
  uint32_t crash_count, crash_window;
  uint32_t ev_cap, ev_stride;      // per-lane pool capacity and scratch stride (u32 words)
  // random delivery (variant 2): Bernoulli + fix-up sampler with p = rd_a / 16 and
  // rd_b-bit index fields; rd_a = 0 selects Floyd (oracle_delivery_bernoulli)
  uint32_t rd_a, rd_b;
  uint32_t rd_rows;                // Bernoulli sampler: bitset rows per lane, max(ceil(m/32), 2^rd_b / 32)
  uint64_t ev_lanes;               // lanes the scratch buffer holds
  uint32_t *scratch;               // [ev_lanes][ev_stride]
  // matrix-core kernel (variant 7, KIND > 0): trials that do not halt in round 1,
  // as offsets within the launch: wave w writes them to its segment
  // defer_seg[w * defer_seg_cap ...], then appends them to defer_list
  // (capacity trial_count) at defer_len
  uint32_t *defer_list, *defer_len, *defer_seg;
  uint32_t defer_seg_cap;
  // per-plan device flag word, set (atomic OR) when a launch broke a capacity
  // invariant -- bit 0: an owner deferred more than defer_seg_cap trials (its
  // extra trials are dropped); bit 1: an event-level message pool filled up.
  // The launch's histogram is then incomplete; bo_plan_check / bo_plan_run
  // report BO_ERR_INTERNAL.
  uint32_t *overflow;
  // event level, N > kMaxEventN (benor_event_big.hip): explicit /stop schedule
  // as (event << 12 | node), ascending
  const uint64_t *ev_stops;
  uint32_t ev_nstops;
  // event level, N > kMaxEventN: a random /stop schedule (crash_at NULL,
  // crash_count > 0) drawn per trial on the device -- its length min(crash_count, m)
  uint32_t ev_rstops;
  // live run (bo_consensus_start_live): the wave-per-trial event kernel at any
  // N, polling a host-mapped mailbox for GET /stop requests served while it
  // runs -- live_box[0] request sequence, [kLiveReq ..) requested-stop bits,
  // [kLiveEv + i] the delivery count at which node i's stop landed (device)
  uint32_t live;
  uint32_t *live_box;
  // event level: run the workgroup-batched kernel (benor_event_live.hip) --
  // live runs, and batch plans under BENOR_EVENT_FORM=wg
  uint32_t ev_wg;
  // diagnostics (BENOR_EVENT_STATS): that kernel's per-batch counters and
  // cycle split, 24 u64 (device) or nullptr
  unsigned long long *ev_stats;
  uint32_t ev_hs;                  // its LDS hash slots per batch (a power of two; set at launch)
  // W kernel trial-list mode: run the trials trial_begin + trial_list[i],
  // i < min(*trial_list_len, trial_count), instead of a contiguous range
  const uint32_t *trial_list, *trial_list_len;
  // matrix-core continuation pass (KIND > 0): cont_round = r >= 2 runs
  // round r of the trials trial_begin + trial_list[i], i < *trial_list_len,
  // which tied in every round before r (x = their round r-1 coins); 0: round 1
  uint32_t cont_round;
  // diagnostics (BENOR_TIMELINE=<file>, packed matrix-core kernel): per wave,
  // kTimelineWords u64 -- wall-clock stamps of its phases and its batch counts
  unsigned long long *timeline;
};

constexpr uint32_t kTimelineWords = 12;


// The live run's host-mapped mailbox (u32 words):
constexpr uint32_t kLiveReq = 2;                 // request bitset words (BO_MAX_N / 32), GET /stop posted
constexpr uint32_t kLiveEv = kLiveReq + 128;     // per-node stop delivery counts (device writes)
constexpr uint32_t kSnapReq = kLiveEv + BO_MAX_N;   // GET /getState snapshot requests (host increments)
constexpr uint32_t kSnapSeq = kSnapReq + 1u;     // the last request served (device writes, after the snapshot)
constexpr uint32_t kSnapE = kSnapSeq + 1u;       // u64: the delivery count the snapshot reflects
constexpr uint32_t kSnapSt = kSnapE + 4u;        // [BO_MAX_N] {killed | x << 8 | decided << 16, k}: the snapshot
constexpr uint32_t kLiveBoxWords = kSnapSt + 2u * BO_MAX_N;

constexpr uint32_t kMfmaContRounds = 3;       // matrix-core passes up to round 3, then the popcount kernel
// The deferral buffer's 64-word length block: pass r's list length at 16 (r - 1).
static_assert(16u * kMfmaContRounds <= 64u, "deferral length words overflow their block");

constexpr uint64_t kDeferChunk = 1ull << 22;   // trials per matrix-core launch when trials can be deferred

// Environment knobs (benor_runtime.cpp kKnobs: the only getenv in the library).
// Each is documented in DESIGN.md §6 and mirrored by benor.KNOBS; none is
// needed in production, every one of them only forces a choice the planner
// makes by itself, for tests, tuning sweeps and diagnostics -- bench.py
// refuses to report with any set.  knob() returns NULL when unset.
const char *knob(const char *name);
uint32_t knob_u32(const char *name, uint32_t dflt);
bool knob_is(const char *name, const char *value);

// Pick the tally block size G and fill nblocks / LDS sizes.
void plan_geometry(KParams &p);

hipError_t launch_lockstep(const KParams &p, int grid_blocks, hipStream_t stream);

// Random delivery, Bernoulli + fix-up sampler (benor_random.hip, r04).
uint32_t random_bern_rows(uint32_t m, uint32_t b);
hipError_t launch_random_bern(const KParams &p, int grid_blocks, hipStream_t stream);

// Event level for kMaxEventN < N <= BO_MAX_N (benor_event_big.hip): one wave per trial.
// The wave-per-trial event kernel keeps its message pool in LDS when it is at
// most this many bytes (4N^2 + 64 u32: N <= 78).
constexpr uint64_t kEventBigLdsPool = 96u * 1024u;
bool event_big_lds_pool(const KParams &p);
uint32_t event_big_lds_bytes(const KParams &p);
hipError_t launch_event_big(const KParams &p, int grid_blocks, hipStream_t stream);

// Workgroup-batched event kernel (benor_event_live.hip, r06): one trial per
// workgroup of a control wave and 1, 3, 7 or 15 event waves; live runs (mailbox
// /stop, /getState snapshots) and single-trial network runs.
uint32_t event_wg_waves(const KParams &p);
// ... and, with no random /stop schedule and no forced wave count, its
// one-wave forms: for N <= kEventRegMaxN the pool, inboxes and node state in
// registers, one event per step (event_reg_regs: pool VGPRs, 0 = not this
// form); for N <= kEventWaveMaxN micro-batches of up to 64 events, the pool
// in LDS (BENOR_EVENT_FORM=wave: this form below kEventRegMaxN too).
constexpr uint32_t kEventRegMaxN = 16;            // the LDS micro-batch form is faster from N ~ 20
constexpr uint32_t kEventWaveMaxN = 64;
uint32_t event_reg_regs(const KParams &p);
bool event_wave_form(const KParams &p);
uint32_t event_wave_lds_bytes(const KParams &p);
bool event_wg_lds_pool(const KParams &p);
uint32_t event_wg_lds_bytes(const KParams &p, uint32_t waves);
hipError_t launch_event_wg(const KParams &p, int grid_blocks, hipStream_t stream);

// Per-shape launchers, explicitly instantiated in benor_w_*.hip (W = 1..32)
// and benor_blocked.hip (G = 11..22).
template <int W>
hipError_t launch_w(const KParams &p, int grid_blocks, hipStream_t stream);
template <int G>
hipError_t launch_b(const KParams &p, int grid_blocks, hipStream_t stream);
// Lane kernel (benor_lane.h), m = 1..kMaxLaneM, instantiated in benor_lane_*.hip.
template <int MM>
hipError_t launch_lane_m(const KParams &p, int grid_blocks, hipStream_t stream);

// Packed matrix-core kernel (benor_mfma_small.h), m = 2..32, benor_mfma_small_02_32.hip.
template <int MM>
hipError_t launch_mfma_small_m(const KParams &p, int grid_blocks, hipStream_t stream);
constexpr uint32_t small_slots(uint32_t m) { return (32u / m) < 8u ? (32u / m) : 8u; }
constexpr uint32_t kSmallMaxRound = 3;   // rounds on the matrix cores; a later tie -> the lane path
// Shared-init Philox passes of a fresh batch: its 64 S trials (from any start
// offset mod 4) use at most 16 S + 1 blocks of stream 1, drawn 64 per pass.
constexpr uint32_t small_init_passes(uint32_t m) { return (16u * small_slots(m) + 1u + 63u) / 64u; }
// LDS words per wave: round-2 and round-3 lists (2 batches each), the round-3
// list's carried x words (2 batches), the lane-path queue (a batch + 64), the
// fresh batch's init blocks (4 words per block)
constexpr uint32_t small_wave_words(uint32_t m) {
  return 7u * 64u * small_slots(m) + 64u + 256u * small_init_passes(m);
}
constexpr uint64_t kSmallMinTrials = 500000;    // shorter packed-shape launches run on the lane kernel
bool small_on_lane(const KParams &p);

// Matrix-core kernel (benor_mfma.h), W = 2..16, instantiated in benor_mfma_*.hip;
// W = 17..64 (m <= 4096): the big-network form, benor_mfma_big.hip.
template <int W>
hipError_t launch_mfma(const KParams &p, int grid_blocks, hipStream_t stream);
hipError_t launch_mfma_big(const KParams &p, int grid_blocks, hipStream_t stream);
uint32_t mfma_big_lds_bytes(const KParams &p, uint32_t block_waves);   // dynamic LDS of one workgroup of the big form
uint32_t mfma_big_block_waves(const KParams &p);                       // its waves per workgroup (1, 2 or 4)
// Workgroup-cooperative big-network form (benor_mfma_coop.hip): the waves of a
// workgroup share one 32-trial group; deferral segments are per workgroup.
bool mfma_big_coop(const KParams &p);                                   // this big-network launch runs it
hipError_t launch_mfma_coop(const KParams &p, int grid_blocks, hipStream_t stream);
uint32_t mfma_coop_lds_bytes(const KParams &p);
uint32_t mfma_coop_block_waves(const KParams &p);                      // 4 or 8
int mfma_coop_blocks_per_cu(const KParams &p);                         // resident workgroups per CU (occupancy)

// Grid size that fills the current device for this configuration, in
// workgroups of block_waves(p) waves.
int lockstep_grid(const KParams &p, int device);
uint32_t block_waves(const KParams &p);
// Owners of deferral segments in a launch of `grid` workgroups: one per wave,
// or one per workgroup in the cooperative big-network form.
uint64_t defer_units(const KParams &p, int grid);

// Matrix-core microbenchmark: e2m1 32x32x64 multiply-adds executed per launch.
hipError_t launch_mfma_peak(float *sink, int grid_blocks, int iters, hipStream_t stream, double *terms_per_launch);

// v_bcnt_u32_b32 microbenchmark: popcount words executed per launch.
hipError_t launch_popc_peak(uint32_t *sink, int grid_blocks, int iters, hipStream_t stream,
                            double *words_per_launch);

}  // namespace benor
