/*
 * benor.h -- C ABI of the MI355X-native Ben-Or consensus simulator (libbenor.so).
 *
 * This is the drop-in boundary for the reference's hot path
 * (viviendbk/ben-or-consensus-algorithm, src/nodes/node.ts:43-163, the
 * POST /message round loop).  Each entry point names the reference interface
 * it replaces.  Plain C types only: pointers, sizes, integers.  No torch or
 * HIP types appear in any signature; streams are passed as `void*`
 * (a hipStream_t, NULL = default stream).
 *
 * Value encoding (src/types.ts:1-8, `Value = 0 | 1 | "?"`):
 *     int8  0 -> 0,  1 -> 1,  2 -> "?",  -1 -> null (faulty node's x)
 * `decided`: -1 -> null, 0 -> false, 1 -> true;  `k`: -1 -> null.
 *
 * Threading: every function may be called from any host thread.  Calls on one
 * bo_network handle are serialised by a lock in the handle; bo_consensus_start
 * holds it only to read the start state and to merge the results, so /stop,
 * /getState and /status stay served while its kernel runs (the N-API addon
 * runs it on a worker thread).  bo_network_destroy must not overlap any other
 * call on the handle.  bo_plan_launch is asynchronous on its stream; all other
 * calls are synchronous.
 */
#ifndef BENOR_H
#define BENOR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BENOR_ABI_VERSION 8

/* Return codes.  The first two are the reference's two launch errors. */
enum {
    BO_OK = 0,
    BO_ERR_ARRAYS_DONT_MATCH = 1,   /* launchNodes.ts:10-11  Error("Arrays don't match") */
    BO_ERR_FAULTY_COUNT = 2,        /* launchNodes.ts:12-13  Error("faultyList doesnt have F faulties") */
    BO_ERR_INVALID_ARGUMENT = 3,
    BO_ERR_NO_DEVICE = 4,           /* no gfx950 device visible: the product never falls back to CPU */
    BO_ERR_HIP = 5,
    BO_ERR_OUT_OF_RANGE = 6,        /* node index >= N */
    BO_ERR_UNSUPPORTED = 7,         /* configuration outside what this build simulates */
    BO_ERR_ALREADY_STARTED = 8,     /* second start on one network: its inboxes persist (node.ts:29-30) */
    BO_ERR_INTERNAL = 9             /* a device-side invariant failed: the affected results are invalid */
};

/* Delivery model.  LOCKSTEP is the reference's semantics for its admissible
 * inputs (exactly F crash faults, launchNodes.ts:12-13): every live node
 * receives every live node's message in every phase.
 * RANDOM_DELIVERY generalises to f <= F crashed nodes: in every phase each
 * live receiver tallies the first N-F arrivals, a uniformly random subset of
 * exactly N-F of the N-f live senders drawn from Philox (no
 * reference counterpart -- the reference rejects f != F).  At f == F the two
 * modes give identical results. */
/* EVENT is message-granular: the reference's handler
 * (node.ts:45-158) delivery by delivery, in a seeded random order, with the
 * reference's mid-run GET /stop (node.ts:191-194) applied at scheduled
 * delivery counts.  Exactly F crash-faulty nodes; N <= 4096 (one lane per
 * trial up to N = 256, one wave per trial above).  Both /stop schedules --
 * explicit (crash_at) and random (crash_count, crash_window) -- work at every
 * N <= 4096. */
enum { BO_MODE_LOCKSTEP = 0, BO_MODE_RANDOM_DELIVERY = 1, BO_MODE_EVENT = 2 };

enum { BO_INIT_RANDOM = 0, BO_INIT_FIXED = 1 };

/* Largest network simulated per trial (N <= 4096 live + faulty nodes). */
#define BO_MAX_N 4096u
/* Largest round cap. */
#define BO_MAX_K 1024u

/* NodeState (src/types.ts:1-8), as served by GET /getState (node.ts:197-199). */
typedef struct bo_node_state {
    int8_t killed;    /* 0/1 */
    int8_t x;         /* -1 null, 0, 1, 2 '?' */
    int8_t decided;   /* -1 null, 0, 1 */
    int8_t pad;
    int32_t k;        /* -1 null */
} bo_node_state;

typedef struct bo_network bo_network;

/* ---- network API: one simulated network, the reference's public surface ---- */

/* launchNetwork(N, F, initialValues, faultyList)  (src/index.ts:4-14)
 *   -> launchNodes (src/nodes/launchNodes.ts:4-44).
 * Performs the reference's two validations in its order and returns their
 * codes; on success *out owns host-side node state (node.ts:21-26):
 * faulty -> {killed:1, x:null, decided:null, k:null}; live -> {0, init, 0, 0}.
 * init values: 0, 1 or 2 ('?').  No GPU work happens here. */
int bo_network_create(uint32_t N, uint32_t F,
                      const int8_t *initial_values, uint32_t n_initial_values,
                      const uint8_t *faulty_list, uint32_t n_faulty_list,
                      bo_network **out);

/* startConsensus(N)  (src/nodes/consensus.ts:3-8) -> GET /start on every node
 * (node.ts:167-188), then the POST /message round loop (node.ts:43-163) until
 * every live node has decided or k_max rounds ran -- one HIP kernel launch on
 * the calling thread's current device, synchronous.  `seed` keys the
 * per-node coins (node.ts:111).  Nodes already stopped act as crashed.
 * Runs once per network: the reference's round inboxes (node.ts:29-30) outlive
 * a run, so a second start is not a fresh consensus and returns
 * BO_ERR_ALREADY_STARTED.  A /stop served while the kernel runs takes effect
 * after it: the node keeps its final state and is killed. */
int bo_consensus_start(bo_network *net, uint64_t seed, uint32_t k_max);

/* startConsensus(N) with GET /stop requests that land while consensus runs
 * (node.ts:191-194 served mid-round; from then on the node drops every
 * message, node.ts:45).  stop_after[i] (n_stop_after == N entries) = number
 * of POST /message deliveries, network-wide, after which node i is stopped;
 * UINT32_MAX = not stopped.  Deliveries follow BO_MODE_EVENT's seeded order
 * (trial 0 of `seed`), so a schedule is reproducible.  With every entry
 * UINT32_MAX (or stop_after NULL) this is bo_consensus_start; otherwise the
 * run is message-granular on the event-level kernel (any N <= BO_MAX_N; a
 * schedule whose entries all name killed nodes is bo_consensus_start) and the
 * per-node states are its final ones, scheduled
 * stops included (killed, x / decided / k as of the stop).  The auto-stop and
 * one-start rules of bo_consensus_start apply. */
int bo_consensus_start_sched(bo_network *net, uint64_t seed, uint32_t k_max,
                             const uint32_t *stop_after, uint32_t n_stop_after);

/* startConsensus(N) as the reference runs it (consensus.ts:3-8, node.ts:167-188):
 * GET /start answers before consensus finishes, and GET /stop / GET /getState
 * requests served while it runs land in it (node.ts:191-199, :45).  Launches
 * the event-level kernel (seeded delivery order, trial 0 of `seed`, any
 * N <= BO_MAX_N; one workgroup of 1-15 event waves and a control wave) on its
 * own HIP stream and returns.  While it runs:
 *   - bo_node_stop / bo_consensus_stop also post to a host-mapped mailbox the
 *     kernel polls (every ~20 us): a request is applied before the next
 *     delivery, and that delivery count is recorded (bo_live_stop_events);
 *   - bo_get_state / bo_get_states answer at once from a snapshot the kernel
 *     writes at its next batch boundary (tens of microseconds): every node's
 *     state as of a delivery count, with the killed flag of every /stop already
 *     served (node.ts:191-194 sets it at once);
 *   - bo_status answers from the killed flags.
 * bo_consensus_wait (blocking) or bo_consensus_poll (not) end the run and merge
 * its final states; a request the kernel did not see before it finished is
 * ordered after the run, as for bo_consensus_start.  The one-start and
 * auto-stop rules of bo_consensus_start apply; bo_network_destroy waits for a
 * live run. */
int bo_consensus_start_live(bo_network *net, uint64_t seed, uint32_t k_max);

/* Wait for a live run (bo_consensus_start_live) and merge its final states;
 * BO_OK at once when none is in flight. */
int bo_consensus_wait(bo_network *net);

/* Without blocking: *running_out = 1 while a live run is in flight; once it
 * has ended, its final states are merged (as bo_consensus_wait) and
 * *running_out = 0. */
int bo_consensus_poll(bo_network *net, int *running_out);

/* After bo_consensus_wait: for each node, the delivery count at which a live
 * run applied its GET /stop, UINT32_MAX if it applied none (n == N).  Passed as
 * bo_consensus_start_sched's stop_after on a fresh network of the same launch,
 * with the same seed, it reproduces the live run exactly (counts below
 * UINT32_MAX - 1). */
int bo_live_stop_events(const bo_network *net, uint32_t *events_out, uint32_t n);

/* stopConsensus(N)  (consensus.ts:10-15) -> GET /stop on every node (node.ts:191-194). */
int bo_consensus_stop(bo_network *net);

/* GET /stop on one node (node.ts:191-194): killed = true (and, during a live
 * run, posted to the running kernel). */
int bo_node_stop(bo_network *net, uint32_t node);

/* GET /getState (node.ts:197-199): the node's current state, answered at once
 * (during a live run: from a snapshot, see bo_get_states). */
int bo_get_state(const bo_network *net, uint32_t node, bo_node_state *out);

/* GET /getState on every node at once (__test__/tests/utils.ts:14-20), out[n],
 * n == N.  During a live run: one snapshot of the running kernel, taken at a
 * batch boundary after *events_out POST /message deliveries -- exactly oracle
 * (iii) truncated there, plus the killed flags of /stop requests served but
 * not yet applied; a snapshot taken within the last 500 us answers later
 * requests too (N concurrent GET /getState cost one).  Otherwise the
 * network's states and *events_out = UINT64_MAX.  events_out may be NULL. */
int bo_get_states(const bo_network *net, bo_node_state *out, uint32_t n, uint64_t *events_out);

/* GET /status (node.ts:33-39): returns 500 ("faulty") or 200 ("live"), or a
 * negative BO_ERR_* code. */
int bo_status(const bo_network *net, uint32_t node);

uint32_t bo_network_size(const bo_network *net);

/* server.close() for every server (benorconsensus.test.ts:14-29). */
void bo_network_destroy(bo_network *net);

/* ---- batch API: many independent trials of one network shape ---- */

typedef struct bo_trials_cfg {
    uint32_t N, F;            /* network size; fault parameter (quorum N-F, decide on > F) */
    uint32_t k_max;           /* round cap, 1..BO_MAX_K */
    uint32_t init_mode;       /* BO_INIT_RANDOM: iid Bernoulli(1/2) per live node; BO_INIT_FIXED */
    uint32_t mode;            /* BO_MODE_LOCKSTEP or BO_MODE_RANDOM_DELIVERY */
    uint32_t reserved;
    uint64_t seed;            /* Philox4x32-10 key */
    const uint8_t *faulty;    /* host [N]; exactly F set (LOCKSTEP, EVENT), at most F (RANDOM_DELIVERY) */
    const int8_t *init;       /* host [N]; used when init_mode == BO_INIT_FIXED */
    /* EVENT mode only: GET /stop schedule.  crash_at[i] = number of deliveries
     * after which node i is stopped (UINT32_MAX = never), or, when crash_at is
     * NULL, crash_count distinct live nodes stopped at uniform delivery counts
     * in [0, crash_window), drawn per trial from Philox. */
    const uint32_t *crash_at; /* host [N] or NULL */
    uint32_t crash_count;
    uint32_t crash_window;
} bo_trials_cfg;

/* Histogram length for a round cap: (k_max + 1) * 3 + 1 uint64 bins.
 *   bin[R*3 + v], 1 <= R <= k_max : every live node decided after round R, common x = v
 *                                   (v = 2: decided values differ)
 *   bin[0*3 + v]                  : not every live node decided within k_max rounds;
 *                                   v = common x, or 2 if they differ
 *   bin[(k_max+1)*3]              : trials whose decided values differ (agreement violations) */
uint32_t bo_hist_len(uint32_t k_max);

typedef struct bo_plan bo_plan;

/* Validate a trial configuration and upload its tables to the current device. */
int bo_plan_create(const bo_trials_cfg *cfg, bo_plan **out);

/* Run global trial ids [trial_begin, trial_begin + trial_count) and ADD their
 * outcomes into hist_dev (device pointer, bo_hist_len(k_max) uint64).
 * Asynchronous on `stream` (hipStream_t or NULL).  A plan owns per-plan
 * device scratch (the matrix-core kernels' deferred-trial lists, the event
 * mode's message pools), so launches of ONE plan must be issued from one host
 * thread at a time and ordered on one stream (or separated by a
 * synchronisation); concurrent launches need one plan each. */
int bo_plan_launch(bo_plan *plan, uint64_t trial_begin, uint64_t trial_count,
                   uint64_t *hist_dev, void *stream);

/* Same, blocking, host histogram (added into hist_host).  Includes bo_plan_check. */
int bo_plan_run(bo_plan *plan, uint64_t trial_begin, uint64_t trial_count, uint64_t *hist_host);

/* Synchronise the device and report device-side invariant failures of this
 * plan's launches since the last check: BO_ERR_INTERNAL when a matrix-core
 * launch deferred more trials than its segment holds (their outcomes are then
 * missing from the histogram).  No reference counterpart: call it after a
 * series of bo_plan_launch before trusting their histograms. */
int bo_plan_check(bo_plan *plan);

/* The roofline's algorithmic unit: VALU popcount words that the per-receiver
 * tallies of one live node-round need, m = live nodes, M = m - (number of "?"
 * initial values) binary votes.  LOCKSTEP / EVENT: the R-phase counts c1
 * (c0 = M - c1); the P-phase counts c1 when M is odd (no tie, so no "?"
 * proposal: c0 = m - c1) and c0, c1 otherwise -- 2 or 3 x ceil(m/32).
 * RANDOM_DELIVERY: both values in both phases, 4 x ceil(m/32). */
uint64_t bo_plan_popc_words_per_node_round(const bo_plan *plan);
uint32_t bo_plan_live_nodes(const bo_plan *plan);

/* Kernel families.  BO_KERNEL_MFMA counts inboxes on the matrix cores
 * (e2m1 operands, exact f32 sums): lockstep, 64 < m <= 1024, m odd, an even
 * number of "?" initial values and m > 2F -- every trial halts in round 1.
 * Its roofline unit is receiver-sender terms, 2m per live node-round. */
enum {
  BO_KERNEL_NONE = -1, /* no live node: outcomes need no kernel */
  BO_KERNEL_BLOCKED = 0,
  BO_KERNEL_W = 1,
  BO_KERNEL_RANDOM = 2,
  BO_KERNEL_EVENT = 4,  /* event level: one lane per trial (N <= 256), one wave per trial (N > 256, live runs) */
  BO_KERNEL_LANE = 6,
  BO_KERNEL_MFMA = 7,
  BO_KERNEL_MFMA_SMALL = 8 /* packed matrix-core kernel: 2 <= m <= 32, m > F, no "?" initial value;
                              64 * min(32/m, 8) trials per wave iteration, block-diagonal e2m1 products;
                              launches of fewer than 5 * 10^5 trials run the lane kernel
                              (BENOR_SMALL_MIN_TRIALS overrides) */
};

/* The kernel family bo_plan_launch runs for this plan.  (The per-node-state
 * launch behind the network API runs the W kernel for an MFMA shape and the
 * lane kernel for an MFMA_SMALL shape.) */
int bo_plan_kernel(const bo_plan *plan);

/* The same choice for a configuration, made on the host (no device needed):
 * *kernel_out = BO_KERNEL_* (BO_KERNEL_NONE for no live node).  Returns
 * bo_plan_create's validation error for an invalid cfg. */
int bo_kernel_for(const bo_trials_cfg *cfg, int *kernel_out);

void bo_plan_destroy(bo_plan *plan);

/* One-shot convenience: create plan, run trial ids [trial_begin, +trial_count), destroy. */
int bo_run_trials(const bo_trials_cfg *cfg, uint64_t trial_begin, uint64_t trial_count,
                  uint64_t *hist_host);

/* Per-node final states of one trial (trial id `trial`), nodes_out[N]. */
int bo_run_trial_states(const bo_trials_cfg *cfg, uint64_t trial, bo_node_state *nodes_out,
                        uint32_t *rounds_out);

/* ---- diagnostics ---- */

/* Time the v_bcnt_u32_b32 peak microbenchmark: returns popcount words/s
 * measured on the current device over `iters` launches (0 on error). */
double bo_popc_peak(uint32_t iters);

/* Time the matrix-core peak microbenchmark (v_mfma_scale_f32_32x32x64_f8f6f4,
 * e2m1 operands, the BO_KERNEL_MFMA instruction): multiply-adds per second on
 * the current device over `iters` launches (0 on error). */
double bo_mfma_peak(uint32_t iters);

/* Message of the last error on this thread ("" if none). */
const char *bo_last_error(void);

int bo_abi_version(void);

/* Digest of the kernel sources this library was built from (16 hex digits).
 * Profiles record it, so a measured figure is only quoted for the same kernels. */
const char *bo_kernel_version(void);

#ifdef __cplusplus
}
#endif

#endif /* BENOR_H */
