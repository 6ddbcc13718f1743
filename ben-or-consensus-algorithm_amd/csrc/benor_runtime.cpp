// benor_runtime.cpp -- C ABI (include/benor.h) over the gfx950 kernels.
//
// Host-side mirror of the reference's network layer:
//   launchNetwork / launchNodes   src/index.ts:4-14, src/nodes/launchNodes.ts:4-44
//   startConsensus / stopConsensus src/nodes/consensus.ts:3-15
//   GET /status, /start, /stop, /getState   src/nodes/node.ts:33-39, :167-199
// The POST /message round loop (node.ts:43-163) runs on the device
// (benor_kernels.hip).  There is no CPU fallback: without a gfx950 device
// every compute entry point returns BO_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <algorithm>
#include <utility>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <thread>
#include <chrono>
#include <vector>

#include "benor.h"
#include "benor_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char *what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return BO_ERR_HIP;
}

#define HIP_TRY(expr)                                  \
  do {                                                 \
    hipError_t e_ = (expr);                            \
    if (e_ != hipSuccess) return hip_fail(e_, #expr);  \
  } while (0)

// The product runs only on a gfx950 device.
int check_device(int *dev_out) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
    return fail(BO_ERR_NO_DEVICE, "no HIP device visible (libbenor has no CPU fallback)");
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, dev));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(BO_ERR_NO_DEVICE, std::string("device is ") + prop.gcnArchName + ", libbenor targets gfx950");
  if (dev_out) *dev_out = dev;
  return BO_OK;
}

__global__ void add_bin_kernel(unsigned long long *hist, uint32_t bin, unsigned long long n) {
  if (threadIdx.x == 0 && blockIdx.x == 0) hist[bin] += n;
}

}  // namespace

namespace benor {
// Every environment knob the library reads.  Production needs none: each
// forces a choice the planner makes by itself (DESIGN.md §6 "knobs").
//   validation: run another product kernel or form on the same trials, so
//     tests can check each against the others and the oracle;
//   tuning: grid shape only (every test checks that the histogram does not
//     depend on it);
//   test: provoke an error path;  diagnostic: instrumented launches.
struct KnobSpec {
  const char *name, *kind;
};
constexpr KnobSpec kKnobs[] = {
    {"BENOR_NO_MFMA", "validation"},            // "1": popcount kernels instead of the matrix-core ones
    {"BENOR_NO_MFMA_BIG", "validation"},        // "1": popcount kernels for m > 1024
    {"BENOR_BIG_FORM", "validation"},           // "wave" / "coop": big-network matrix-core form
    {"BENOR_COOP_BW", "validation"},            // 4 / 8: waves per cooperative workgroup
    {"BENOR_SMALL_MIN_TRIALS", "validation"},   // packed matrix-core kernel from this launch size
    {"BENOR_BLOCKS_PER_CU", "tuning"},          // workgroups per CU (grid)
    {"BENOR_EVENT_LANES_PER_CU", "tuning"},     // event level, N <= 256: lanes per CU
    {"BENOR_EVENT_FORM", "validation"},         // "wg": batch event plans on the workgroup-batched kernel
    {"BENOR_LIVE_WAVES", "tuning"},             // 1 / 3 / 7 / 15: event waves of the workgroup-batched kernel
    {"BENOR_EVENT_STATS", "diagnostic"},        // workgroup-batched kernel: batch counters and cycle split to a file
    {"BENOR_TEST_DEFER_SEG_CAP", "test"},       // deferral segment capacity below the sizing rule
    {"BENOR_TIMELINE", "diagnostic"},           // packed matrix-core kernel: per-wave phase stamps to a file
};

const char *knob(const char *name) {
  for (const KnobSpec &k : kKnobs)
    if (std::strcmp(k.name, name) == 0) return std::getenv(name);
  std::fprintf(stderr, "libbenor: knob %s is not registered in kKnobs\n", name);
  std::abort();
}

uint32_t knob_u32(const char *name, uint32_t dflt) {
  const char *v = knob(name);
  return v && *v ? (uint32_t)std::strtoul(v, nullptr, 10) : dflt;
}

bool knob_is(const char *name, const char *value) {
  const char *v = knob(name);
  return v && std::strcmp(v, value) == 0;
}
}  // namespace benor

// One simulated network.  `mu` guards the node states: bo_consensus_start may
// run on a worker thread (the N-API addon's napi_async_work) while the caller's
// thread serves /stop, /getState and /status.  The kernel runs without the
// lock; its results are merged under it.
struct bo_live;
struct bo_network {
  uint32_t N = 0, F = 0;
  std::vector<bo_node_state> st;
  std::vector<uint8_t> faulty;
  bool started = false;     // GET /start was served (node.ts:167-188); inboxes persist after it
  bool in_flight = false;   // a start's kernel is running
  std::shared_ptr<bo_live> live;   // a live run (bo_consensus_start_live) not yet finalized
  int live_rc = 0;          // the result of the last live run finalized
  std::vector<uint32_t> stop_events;   // its /stop delivery counts, after the run
  mutable std::mutex mu;
  std::mutex wait_mu;       // serialises the end of a live run (live_finalize)
  std::mutex snap_mu;       // one GET /getState snapshot request in flight at a time
};

struct bo_plan {
  benor::KParams kp{};
  bo_trials_cfg cfg{};
  std::vector<uint32_t> live_ids;
  uint32_t *d_live = nullptr;
  uint4 *d_init = nullptr;
  int8_t *d_init_x = nullptr;      // event mode
  uint32_t *d_crash = nullptr;     // event mode
  uint32_t *d_scratch = nullptr;   // event mode
  uint32_t *d_defer = nullptr;     // matrix-core KIND > 0: deferred-trial list, its length, per-wave segments
  uint64_t defer_words = 0;
  uint32_t *d_flag = nullptr;      // KParams::overflow (bo_plan_check)
  uint64_t *d_stops = nullptr;     // event level, N > 256: sorted /stop schedule
  int device = 0;
};

namespace {
// The resources of one single-trial event-level run, kept for the next one
// (r05: the default startConsensus is a live run, and a network of the
// reference's size spent 0.8 ms of its 0.83 ms creating a stream, pinning a
// mailbox and allocating and freeing ten device buffers).  A slot is one
// device's stream, a host-mapped mailbox for BO_MAX_N nodes (GET /stop
// requests, their landing points, GET /getState snapshots) and one device
// buffer that grows to the largest run it served.  Slots are handed out under
// a lock and returned when their run ends; a buffer above kSlotKeepBytes is
// freed on return (a process that once ran a large network does not keep its
// message pool), and a slot whose run failed is destroyed, not reused.
struct LiveSlot {
  int device = -1;
  hipStream_t s = nullptr;
  uint32_t *box = nullptr;             // host-mapped mailbox (benor::kLiveReq .. kLiveBoxWords layout)
  uint32_t *dbox = nullptr;            // its device address
  unsigned char *d = nullptr;          // flag | states | hist | rounds | live ids | init x | stops | pool
  size_t bytes = 0;
  // pinned host copy of the buffer's head: the upload reads it, and the
  // result head (flag | states | hist | rounds) is copied back into it right
  // behind the kernel, so the end of a run is one stream synchronisation
  unsigned char *hp = nullptr;
  size_t hp_bytes = 0;
};
constexpr size_t kSlotKeepBytes = 64u << 20;
std::mutex g_slots_mu;
std::vector<LiveSlot *> g_free_slots;

// Where the run's results sit in the slot's buffer.
struct WgRun {
  size_t o_st = 0, o_r = 0;            // states [N], round word (the head read back ends after it)
  size_t o_stats = 0;                  // BENOR_EVENT_STATS counters (24 u64, after the round word)
  uint32_t N = 0, F = 0;
};
}  // namespace

// A live run (bo_consensus_start_live): the workgroup-batched event kernel
// (benor_event_live.hip) runs on its slot's stream while the caller serves
// /stop, /getState and /status; GET /stop requests and /getState snapshot
// requests reach the running kernel through the slot's mailbox.  Shared by the
// network and by every caller that reads its mailbox (snapshots), so the slot
// goes back to the pool only when the last of them is done.
struct bo_live {
  LiveSlot *slot = nullptr;
  WgRun run;
  std::vector<uint32_t> active;        // the nodes that run
  bool failed = false;                 // the run's stream reported an error: the slot is not reused
  // the last /getState snapshot (under bo_network::snap_mu): the kernel's
  // words of the active nodes, its delivery count and when it was served
  std::vector<uint32_t> snap_words;
  uint64_t snap_e = 0;
  std::chrono::steady_clock::time_point snap_t{};
  bool snap_ok = false;
  ~bo_live();
};

namespace {
// Post GET /stop requests to a live run (caller holds net->mu): the nodes'
// request bits (one OR per 32-node word), then the sequence word.  The
// kernel's control wave applies the bits it reads in the poll after the one
// that saw the new sequence, so one call's requests land together.
void live_post(bo_live *lr, const uint32_t *ids, uint32_t n) {
  uint32_t *box = lr->slot->box;
  uint32_t words[BO_MAX_N / 32] = {};
  for (uint32_t j = 0; j < n; ++j) words[ids[j] >> 5] |= 1u << (ids[j] & 31u);
  for (uint32_t w = 0; w < BO_MAX_N / 32; ++w)
    if (words[w]) __atomic_fetch_or(&box[benor::kLiveReq + w], words[w], __ATOMIC_RELAXED);
  __atomic_fetch_add(&box[0], 1u, __ATOMIC_RELEASE);
}
}  // namespace

extern "C" {

const char *bo_last_error(void) { return g_err.c_str(); }
int bo_abi_version(void) { return BENOR_ABI_VERSION; }
#ifndef BENOR_KERNEL_SHA
#define BENOR_KERNEL_SHA "unknown"
#endif
const char *bo_kernel_version(void) { return BENOR_KERNEL_SHA; }
uint32_t bo_hist_len(uint32_t k_max) { return (k_max + 1u) * 3u + 1u; }

// ------------------------------------------------------------ network API
int bo_network_create(uint32_t N, uint32_t F, const int8_t *init, uint32_t n_init,
                      const uint8_t *faulty, uint32_t n_faulty, bo_network **out) {
  if (!out) return fail(BO_ERR_INVALID_ARGUMENT, "out is NULL");
  *out = nullptr;
  // launchNodes.ts:10-11
  if (n_init != n_faulty || N != n_init) return fail(BO_ERR_ARRAYS_DONT_MATCH, "Arrays don't match");
  if (N > 0 && (!init || !faulty)) return fail(BO_ERR_INVALID_ARGUMENT, "initial_values / faulty_list is NULL");
  uint32_t cnt = 0;
  for (uint32_t i = 0; i < n_faulty; ++i) cnt += faulty[i] ? 1u : 0u;
  // launchNodes.ts:12-13
  if (cnt != F) return fail(BO_ERR_FAULTY_COUNT, "faultyList doesnt have F faulties");
  if (N > BO_MAX_N) return fail(BO_ERR_UNSUPPORTED, "N exceeds BO_MAX_N");
  for (uint32_t i = 0; i < N; ++i)
    if (init[i] < 0 || init[i] > 2) return fail(BO_ERR_INVALID_ARGUMENT, "initial value must be 0, 1 or '?'(2)");
  auto *net = new bo_network();
  net->N = N;
  net->F = F;
  net->st.resize(N);
  net->faulty.assign(faulty, faulty + N);
  for (uint32_t i = 0; i < N; ++i) {   // node.ts:21-26
    const bool f = faulty[i] != 0;
    net->st[i].killed = f ? 1 : 0;
    net->st[i].x = f ? -1 : init[i];
    net->st[i].decided = f ? -1 : 0;
    net->st[i].pad = 0;
    net->st[i].k = f ? -1 : 0;
  }
  *out = net;
  return BO_OK;
}

uint32_t bo_network_size(const bo_network *net) { return net ? net->N : 0u; }

void bo_network_destroy(bo_network *net) {
  if (!net) return;
  (void)bo_consensus_wait(net);   // a live run still holds device buffers
  delete net;
}

int bo_status(const bo_network *net, uint32_t i) {   // node.ts:33-39
  if (!net) return -fail(BO_ERR_INVALID_ARGUMENT, "net is NULL");
  if (i >= net->N) return -fail(BO_ERR_OUT_OF_RANGE, "node index out of range");
  std::lock_guard<std::mutex> g(net->mu);
  return net->st[i].killed ? 500 : 200;
}

namespace {
int get_states_impl(bo_network *net, bo_node_state *out, uint64_t *events_out);
}  // namespace

// GET /getState answers at once with the node's current state (node.ts:197-199):
// during a live run, from a snapshot the kernel takes at its next batch
// boundary (bo_get_states).
int bo_get_state(const bo_network *net, uint32_t i, bo_node_state *out) {   // node.ts:197-199
  if (!net || !out) return fail(BO_ERR_INVALID_ARGUMENT, "NULL argument");
  if (i >= net->N) return fail(BO_ERR_OUT_OF_RANGE, "node index out of range");
  {
    std::lock_guard<std::mutex> g(net->mu);
    if (!net->live) {
      *out = net->st[i];
      return net->live_rc;
    }
  }
  std::vector<bo_node_state> all(net->N);
  const int rc = get_states_impl(const_cast<bo_network *>(net), all.data(), nullptr);
  *out = all[i];
  return rc;
}

int bo_node_stop(bo_network *net, uint32_t i) {   // node.ts:191-194
  if (!net) return fail(BO_ERR_INVALID_ARGUMENT, "net is NULL");
  if (i >= net->N) return fail(BO_ERR_OUT_OF_RANGE, "node index out of range");
  std::lock_guard<std::mutex> g(net->mu);
  net->st[i].killed = 1;
  if (net->live) live_post(net->live.get(), &i, 1u);
  return BO_OK;
}

int bo_consensus_stop(bo_network *net) {   // consensus.ts:10-15
  if (!net) return fail(BO_ERR_INVALID_ARGUMENT, "net is NULL");
  std::lock_guard<std::mutex> g(net->mu);
  for (auto &s : net->st) s.killed = 1;
  if (net->live) {
    std::vector<uint32_t> all(net->N);
    for (uint32_t i = 0; i < net->N; ++i) all[i] = i;
    live_post(net->live.get(), all.data(), net->N);
  }
  return BO_OK;
}

int bo_consensus_start(bo_network *net, uint64_t seed, uint32_t k_max) {   // consensus.ts:3-8
  return bo_consensus_start_sched(net, seed, k_max, nullptr, 0u);
}

namespace {
// What a GET /start (node.ts:167-188) runs: the nodes not killed, their x, and
// their /stop schedule entries.  `launch` is false when nothing needs a kernel.
struct StartPlan {
  std::vector<uint8_t> crashed;
  std::vector<int8_t> x;
  std::vector<uint32_t> active, sched;
  bool scheduled = false;   // a /stop lands on a node that runs (entries of killed nodes are moot)
  bool launch = false;
};

int start_prologue(bo_network *net, uint32_t k_max, const uint32_t *stop_after, uint32_t n_stop_after,
                   StartPlan &sp) {
  if (!net) return fail(BO_ERR_INVALID_ARGUMENT, "net is NULL");
  if (k_max < 1 || k_max > BO_MAX_K) return fail(BO_ERR_INVALID_ARGUMENT, "k_max out of range");
  const uint32_t N = net->N;
  if (stop_after && n_stop_after != N) return fail(BO_ERR_INVALID_ARGUMENT, "stop schedule must have N entries");
  sp.crashed.assign(N, 0);
  sp.x.assign(N, 0);
  sp.sched.assign(N, 0xFFFFFFFFu);
  std::lock_guard<std::mutex> g(net->mu);
  // The reference's per-node inboxes (node.ts:29-30) live as long as the
  // server: a second GET /start pushes round-1 messages onto inboxes that
  // already hold them, and every push past N-F re-triggers the tally
  // (node.ts:47-52).  That is not a fresh consensus, so it is refused.
  if (net->started)
    return fail(BO_ERR_ALREADY_STARTED, net->in_flight
                ? "consensus is already running on this network"
                : "consensus already started on this network: node inboxes persist across /start "
                  "(node.ts:29-30), launch a new network to run again");
  // Nodes that run: not killed (faulty from launch, or stopped).  They send
  // and receive; killed nodes do neither (node.ts:45, :171).
  for (uint32_t i = 0; i < N; ++i) {
    sp.crashed[i] = net->st[i].killed ? 1 : 0;
    sp.x[i] = net->st[i].killed ? 0 : net->st[i].x;
    if (!net->st[i].killed) {
      sp.active.push_back(i);
      if (stop_after) sp.sched[i] = stop_after[i];
    }
  }
  for (uint32_t i : sp.active) sp.scheduled = sp.scheduled || sp.sched[i] != 0xFFFFFFFFu;
  if (sp.active.empty()) { net->started = true; return BO_OK; }
  const int64_t quorum = (int64_t)N - (int64_t)net->F;
  // Fewer running senders than the quorum: no R-phase ever triggers
  // (node.ts:52), every running node stays at k = 1, undecided.
  if ((int64_t)sp.active.size() < quorum) {
    for (uint32_t i : sp.active) net->st[i].k = 1;   // node.ts:172
    net->started = true;
    return BO_OK;
  }
  int dev = 0;
  const int rc = check_device(&dev);
  if (rc) return rc;
  net->started = true;
  net->in_flight = true;
  sp.launch = true;
  return BO_OK;
}

bo_trials_cfg start_cfg(const bo_network *net, uint64_t seed, uint32_t k_max, StartPlan &sp, int mode) {
  bo_trials_cfg cfg{};
  cfg.N = net->N;
  cfg.F = net->F;
  cfg.k_max = k_max;
  cfg.init_mode = BO_INIT_FIXED;
  cfg.mode = mode;
  cfg.seed = seed;
  cfg.faulty = sp.crashed.data();
  cfg.init = sp.x.data();
  cfg.crash_at = sp.scheduled ? sp.sched.data() : nullptr;
  return cfg;
}

// The run's final states into the network (caller holds net->mu).  A /stop
// the run applied is part of it (the kernel's killed flag); one served while
// the kernel ran but not applied by it is ordered after it: the node keeps its
// final x / decided / k and stays killed.
void merge_states(bo_network *net, const std::vector<uint32_t> &active, const std::vector<bo_node_state> &states) {
  const uint32_t N = net->N;
  for (uint32_t i : active) {
    const int8_t killed = net->st[i].killed;
    net->st[i] = states[i];
    net->st[i].killed = (int8_t)(killed | states[i].killed);
  }
  // The reference's auto-stop (node.ts:116-145): after its P-phase a node asks
  // every node's /getState and, when every answer has `decided` truthy, sends
  // /stop to all of them.  A faulty node answers decided: null (node.ts:24)
  // and a node stopped before the run answers false, so it fires only when
  // every node of the network decided -- then every node ends killed.
  bool all_decided = true;
  for (uint32_t i = 0; i < N; ++i) all_decided = all_decided && net->st[i].decided == 1;
  if (all_decided)
    for (uint32_t i = 0; i < N; ++i) net->st[i].killed = 1;
}
}  // namespace

namespace {
int run_sched_wg(const bo_trials_cfg *cfg, std::vector<bo_node_state> &states);
}  // namespace

// startConsensus with GET /stop requests landing during the run (node.ts:191-194
// served while the round loop is in flight).  Without a schedule: the lockstep
// round loop (every running node hears every running node).  With
// one: the event-level kernel, delivery by delivery in the seeded order, each
// scheduled /stop applied after its node's delivery count (oracle (iii)).
int bo_consensus_start_sched(bo_network *net, uint64_t seed, uint32_t k_max, const uint32_t *stop_after,
                             uint32_t n_stop_after) {
  StartPlan sp;
  int rc = start_prologue(net, k_max, stop_after, n_stop_after, sp);
  if (rc || !sp.launch) return rc;
  // Launch-time validation is already done; here the crashed set is the
  // killed set, which has exactly N - quorum = F members at this point.
  const bo_trials_cfg cfg = start_cfg(net, seed, k_max, sp, sp.scheduled ? BO_MODE_EVENT : BO_MODE_LOCKSTEP);
  std::vector<bo_node_state> states(net->N);
  uint32_t rounds = 0;
  // a schedule: one trial of the workgroup-batched event kernel; none: the
  // lockstep round loop
  rc = sp.scheduled ? run_sched_wg(&cfg, states) : bo_run_trial_states(&cfg, 0, states.data(), &rounds);
  std::lock_guard<std::mutex> g(net->mu);
  net->in_flight = false;
  if (rc) {
    net->started = false;          // nothing ran: the start may be retried
    return rc;
  }
  merge_states(net, sp.active, states);
  return BO_OK;
}

// -------------------------------------------------------------- batch API
// Validation and kernel planning of a trial configuration, host only: the
// live-node map, the fixed-init plane and the KParams shape (no device fields).
static int plan_host(const bo_trials_cfg *cfg, std::vector<uint32_t> &live, std::vector<uint4> &plane,
                     benor::KParams &kp, bool live_run = false) {
  if (!cfg) return fail(BO_ERR_INVALID_ARGUMENT, "NULL argument");
  if (cfg->N < 1 || cfg->N > BO_MAX_N) return fail(BO_ERR_UNSUPPORTED, "N must be in [1, 4096]");
  if (cfg->k_max < 1 || cfg->k_max > BO_MAX_K) return fail(BO_ERR_INVALID_ARGUMENT, "k_max must be in [1, 1024]");
  if (cfg->mode != BO_MODE_LOCKSTEP && cfg->mode != BO_MODE_RANDOM_DELIVERY && cfg->mode != BO_MODE_EVENT)
    return fail(BO_ERR_UNSUPPORTED, "unknown delivery mode");
  if (cfg->init_mode != BO_INIT_RANDOM && cfg->init_mode != BO_INIT_FIXED)
    return fail(BO_ERR_INVALID_ARGUMENT, "unknown init_mode");
  if (!cfg->faulty) return fail(BO_ERR_INVALID_ARGUMENT, "faulty is NULL");
  if (cfg->init_mode == BO_INIT_FIXED && !cfg->init) return fail(BO_ERR_INVALID_ARGUMENT, "init is NULL");
  uint32_t f = 0;
  for (uint32_t i = 0; i < cfg->N; ++i) f += cfg->faulty[i] ? 1u : 0u;
  // Lockstep = the reference's admissible inputs: exactly F crash faults
  // (launchNodes.ts:12-13).  Random delivery admits f <= F.
  if (cfg->mode != BO_MODE_RANDOM_DELIVERY && f != cfg->F)
    return fail(BO_ERR_FAULTY_COUNT, "faultyList doesnt have F faulties");
  if (cfg->mode == BO_MODE_RANDOM_DELIVERY && f > cfg->F)
    return fail(BO_ERR_FAULTY_COUNT, "random delivery needs at most F crash-faulty nodes");
  live.clear();
  for (uint32_t i = 0; i < cfg->N; ++i)
    if (!cfg->faulty[i]) live.push_back(i);
  const uint32_t m = (uint32_t)live.size();
  kp = benor::KParams{};
  kp.N = cfg->N;
  kp.F = cfg->F;
  kp.m = m;
  kp.W = (m + 63u) / 64u;
  kp.k_max = cfg->k_max;
  kp.init_mode = cfg->init_mode;
  kp.seed = cfg->seed;
  kp.mode = cfg->mode;
  kp.q = cfg->N - cfg->F;
  kp.crash_count = cfg->crash_count;
  kp.crash_window = cfg->crash_window;
  if (cfg->mode == BO_MODE_EVENT && !cfg->crash_at && cfg->crash_count > 0 && cfg->crash_window > 0)
    kp.ev_rstops = std::min<uint32_t>(cfg->crash_count, m);   // per-trial random /stop schedule
  kp.live = live_run && cfg->mode == BO_MODE_EVENT ? 1u : 0u;
  for (uint32_t i = 0; i < cfg->N && i < 4u * 64u; ++i)
    if (cfg->faulty[i]) kp.faulty_mask[i >> 6] |= 1ull << (i & 63u);
  if (m == 0) {
    kp.hist_len = bo_hist_len(cfg->k_max);
    return BO_OK;
  }
  plane.assign(kp.W, make_uint4(0, 0, 0, 0));
  if (cfg->init_mode == BO_INIT_FIXED) {
    uint32_t n0 = 0, n1 = 0;
    for (uint32_t c = 0; c < m; ++c) {
      const int8_t v = cfg->init[live[c]];
      if (v < 0 || v > 2) return fail(BO_ERR_INVALID_ARGUMENT, "initial value must be 0, 1 or '?'(2)");
      const uint32_t w = c >> 6, b = c & 63u;
      uint32_t *r = reinterpret_cast<uint32_t *>(&plane[w]);
      if (v == 0) { r[b >> 5] |= 1u << (b & 31u); ++n0; }
      if (v == 1) { r[2 + (b >> 5)] |= 1u << (b & 31u); ++n1; }
      if (v == 2) ++kp.init_q;
    }
    kp.init_tie = n0 == n1 ? 1u : 0u;
  }
  benor::plan_geometry(kp);   // after init_q: the kernel choice depends on the round-1 vote parity
  return BO_OK;
}

// BO_KERNEL_* of a plan: its variant, except the wave-per-trial event kernel
// (variant 5: N > 256 or a live run), which is the event-level family too.
static int kernel_family(const benor::KParams &kp) {
  if (kp.m == 0) return BO_KERNEL_NONE;
  return kp.variant == 5u ? BO_KERNEL_EVENT : (int)kp.variant;
}

int bo_kernel_for(const bo_trials_cfg *cfg, int *kernel_out) {
  if (!kernel_out) return fail(BO_ERR_INVALID_ARGUMENT, "NULL argument");
  std::vector<uint32_t> live;
  std::vector<uint4> plane;
  benor::KParams kp;
  const int rc = plan_host(cfg, live, plane, kp);
  if (rc) return rc;
  *kernel_out = kernel_family(kp);
  return BO_OK;
}

static int plan_create_impl(const bo_trials_cfg *cfg, bo_plan **out, bool live_run) {
  if (!cfg || !out) return fail(BO_ERR_INVALID_ARGUMENT, "NULL argument");
  *out = nullptr;
  std::vector<uint32_t> live;
  std::vector<uint4> plane;
  benor::KParams kp0;
  int rc = plan_host(cfg, live, plane, kp0, live_run);
  if (rc) return rc;
  int dev = 0;
  rc = check_device(&dev);
  if (rc) return rc;

  auto *pl = new bo_plan();
  pl->cfg = *cfg;
  pl->cfg.faulty = nullptr;
  pl->cfg.init = nullptr;
  pl->cfg.crash_at = nullptr;
  pl->device = dev;
  pl->live_ids = live;
  pl->kp = kp0;
  benor::KParams &kp = pl->kp;
  const uint32_t m = kp.m;
  {
    hipError_t e = hipMalloc(&pl->d_flag, sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(pl->d_flag, 0, sizeof(uint32_t));
    if (e != hipSuccess) { bo_plan_destroy(pl); return hip_fail(e, "plan flag"); }
  }
  if (m > 0) {
    hipError_t e = hipMalloc(&pl->d_live, sizeof(uint32_t) * m);
    if (e == hipSuccess) e = hipMalloc(&pl->d_init, sizeof(uint4) * kp.W);
    if (e == hipSuccess) e = hipMemcpy(pl->d_live, pl->live_ids.data(), sizeof(uint32_t) * m, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(pl->d_init, plane.data(), sizeof(uint4) * kp.W, hipMemcpyHostToDevice);
    if (e != hipSuccess) { bo_plan_destroy(pl); return hip_fail(e, "plan upload"); }
    kp.live_ids = pl->d_live;
    kp.init_plane = pl->d_init;
    if (cfg->mode == BO_MODE_EVENT && kp.variant == 5) {
      // one wave per trial, each with a pool of ev_cap messages: as many
      // concurrent trials as CUs, within ~4 GiB of pools
      std::vector<int8_t> ix(cfg->N, 0);
      if (cfg->init_mode == BO_INIT_FIXED)
        for (uint32_t i = 0; i < cfg->N; ++i) ix[i] = cfg->init[i];
      std::vector<uint64_t> stops;
      if (cfg->crash_at)
        for (uint32_t i = 0; i < cfg->N; ++i)
          if (cfg->crash_at[i] != 0xFFFFFFFFu) stops.push_back(((uint64_t)cfg->crash_at[i] << 12) | i);
      std::sort(stops.begin(), stops.end());
      int cus = 256;
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      const uint64_t slot = (uint64_t)kp.ev_stride * 4u;
      uint64_t slots = std::max<uint64_t>(1u, std::min<uint64_t>((uint64_t)cus, (4ull << 30) / slot));
      if (live_run) slots = 1u;                      // a live run is one trial
      kp.ev_lanes = slots;
      e = hipMalloc(&pl->d_init_x, cfg->N);
      if (e == hipSuccess) e = hipMemcpy(pl->d_init_x, ix.data(), cfg->N, hipMemcpyHostToDevice);
      if (e == hipSuccess && !stops.empty()) {
        e = hipMalloc(&pl->d_stops, sizeof(uint64_t) * stops.size());
        if (e == hipSuccess)
          e = hipMemcpy(pl->d_stops, stops.data(), sizeof(uint64_t) * stops.size(), hipMemcpyHostToDevice);
      }
      if (e == hipSuccess) e = hipMalloc(&pl->d_scratch, slots * slot);
      if (e != hipSuccess) { bo_plan_destroy(pl); return hip_fail(e, "event-mode scratch"); }
      kp.init_x = pl->d_init_x;
      kp.ev_stops = pl->d_stops;
      kp.ev_nstops = (uint32_t)stops.size();
      kp.scratch = pl->d_scratch;
    } else if (cfg->mode == BO_MODE_EVENT) {
      std::vector<int8_t> ix(cfg->N, 0);
      if (cfg->init_mode == BO_INIT_FIXED)
        for (uint32_t i = 0; i < cfg->N; ++i) ix[i] = cfg->init[i];
      // scratch: one slice per lane, at most ~4 GiB
      const uint64_t stride_bytes = (uint64_t)kp.ev_stride * 4u;
      int cus = 256;
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      // Lanes per CU: the mode is bound by the latency of per-lane scratch
      // accesses, so fewer lanes whose slices stay cache-resident beat full
      // occupancy: 512 per CU for slices up to 4 KiB (N <= 12), else 256
      // (tools/ev_sweep.sh, BENOR_EVENT_LANES_PER_CU overrides).
      uint64_t per_cu = benor::knob_u32("BENOR_EVENT_LANES_PER_CU", stride_bytes <= 4096u ? 512u : 256u);
      if (per_cu < 256u) per_cu = 256u;
      uint64_t lanes = (uint64_t)cus * per_cu;
      const uint64_t fit = (4ull << 30) / stride_bytes;
      if (fit < lanes) lanes = fit;
      lanes = lanes / 256u * 256u;
      if (lanes < 256u) lanes = 256u;
      kp.ev_lanes = lanes;
      e = hipMalloc(&pl->d_init_x, cfg->N);
      if (e == hipSuccess) e = hipMemcpy(pl->d_init_x, ix.data(), cfg->N, hipMemcpyHostToDevice);
      if (e == hipSuccess && cfg->crash_at) {
        e = hipMalloc(&pl->d_crash, sizeof(uint32_t) * cfg->N);
        if (e == hipSuccess) e = hipMemcpy(pl->d_crash, cfg->crash_at, sizeof(uint32_t) * cfg->N, hipMemcpyHostToDevice);
      }
      if (e == hipSuccess) e = hipMalloc(&pl->d_scratch, lanes * stride_bytes);
      if (e != hipSuccess) { bo_plan_destroy(pl); return hip_fail(e, "event-mode scratch"); }
      kp.init_x = pl->d_init_x;
      kp.crash_at = pl->d_crash;
      kp.scratch = pl->d_scratch;
    }
  }
  *out = pl;
  return BO_OK;
}

int bo_plan_create(const bo_trials_cfg *cfg, bo_plan **out) { return plan_create_impl(cfg, out, false); }

void bo_plan_destroy(bo_plan *pl) {
  if (!pl) return;
  if (pl->d_live) (void)hipFree(pl->d_live);
  if (pl->d_init) (void)hipFree(pl->d_init);
  if (pl->d_init_x) (void)hipFree(pl->d_init_x);
  if (pl->d_crash) (void)hipFree(pl->d_crash);
  if (pl->d_scratch) (void)hipFree(pl->d_scratch);
  if (pl->d_defer) (void)hipFree(pl->d_defer);
  if (pl->d_flag) (void)hipFree(pl->d_flag);
  if (pl->d_stops) (void)hipFree(pl->d_stops);
  delete pl;
}

uint32_t bo_plan_live_nodes(const bo_plan *pl) { return pl ? pl->kp.m : 0u; }

int bo_plan_kernel(const bo_plan *pl) {
  if (!pl) return -BO_ERR_INVALID_ARGUMENT;
  return kernel_family(pl->kp);
}

// Lockstep: the R-phase needs c1 only (c0 = M - c1, M binary votes,
// node.ts:52,56-62).  The P-phase needs c0 and c1 (node.ts:92-98) unless M
// is odd: then no R-phase count can tie, no proposal is "?" (node.ts:63-69),
// and c0 = m - c1.  So 2 counts of ceil(m/32) words for odd M (the bench's
// m = 683), 3 for even M (round-1 parity: M = m - init_q).  Random delivery
// counts both values in both phases: 4.
uint64_t bo_plan_popc_words_per_node_round(const bo_plan *pl) {
  if (!pl) return 0;
  uint64_t counts = 4ull;
  if (pl->kp.mode != BO_MODE_RANDOM_DELIVERY) counts = ((pl->kp.m - pl->kp.init_q) & 1u) ? 2ull : 3ull;
  return counts * ((pl->kp.m + 31ull) / 32ull);
}

// Diagnostics (BENOR_TIMELINE=<file>): the packed matrix-core kernel stamps
// each wave's phases; one CSV line per wave is appended to the file
// (tools/timeline_report.py).  Synchronous; not for timing the launch itself.
static hipError_t launch_with_timeline(benor::KParams kp, int grid, hipStream_t s, const char *path) {
  const size_t words = (size_t)grid * benor::kWavesPerBlock * benor::kTimelineWords;
  unsigned long long *d = nullptr;
  hipError_t e = hipMalloc(&d, words * sizeof(unsigned long long));
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(d, 0, words * sizeof(unsigned long long), s);
  kp.timeline = d;
  if (e == hipSuccess) e = benor::launch_lockstep(kp, grid, s);
  std::vector<unsigned long long> h(words);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess) e = hipMemcpy(h.data(), d, words * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return e;
  if (FILE *f = std::fopen(path, "a")) {
    std::fprintf(f, "# launch m=%u trials=%llu grid=%d waves=%d\n", kp.m, (unsigned long long)kp.trial_count, grid,
                 grid * benor::kWavesPerBlock);
    for (size_t w = 0; w < (size_t)grid * benor::kWavesPerBlock; ++w) {
      const unsigned long long *t = h.data() + w * benor::kTimelineWords;
      std::fprintf(f, "%zu", w);
      for (uint32_t i = 0; i < 11u; ++i) std::fprintf(f, ",%llu", t[i]);
      std::fprintf(f, "\n");
    }
    std::fclose(f);
  }
  return hipSuccess;
}

static int plan_launch_impl(bo_plan *pl, uint64_t trial_begin, uint64_t trial_count, uint64_t *hist_dev,
                            bo_node_state *node_out, uint32_t *rounds_out, hipStream_t s) {
  if (trial_count == 0) return BO_OK;
  benor::KParams kp = pl->kp;
  if (kp.m == 0) {   // no live node: every trial lands in bin (0, 2)
    hipLaunchKernelGGL(add_bin_kernel, dim3(1), dim3(64), 0, s,
                       reinterpret_cast<unsigned long long *>(hist_dev), 2u, (unsigned long long)trial_count);
    HIP_TRY(hipGetLastError());
    return BO_OK;
  }
  kp.hist = reinterpret_cast<unsigned long long *>(hist_dev);
  kp.overflow = pl->d_flag;
  kp.node_out = node_out;
  kp.rounds_out = rounds_out;
  if (kp.variant == 7 && kp.G > 0u && !node_out && !rounds_out) {
    // Matrix-core round 1 with deferral (benor_mfma.h, KIND > 0): per chunk of
    // at most kDeferChunk trials, the matrix-core launch records the trials
    // that do not halt in round 1, and the W kernel runs exactly those from
    // round 1 (trial-list mode; the list length is read on the device, so
    // the two launches queue back to back with no host sync).
    const uint64_t cap = std::min<uint64_t>(trial_count, benor::kDeferChunk);
    kp.trial_count = cap;
    const int grid = benor::lockstep_grid(kp, pl->device);
    // Continuation passes: a trial that tied in round 1 starts round 2 from its
    // round-1 coins, so the matrix cores run rounds 2 .. kMfmaContRounds of the
    // deferred trials too, each pass deferring its own ties; whatever is left
    // goes to the popcount kernel, which re-runs it from round 1.
    const uint32_t last_round = std::min<uint32_t>(benor::kMfmaContRounds, kp.k_max - 1u);
    // A pass's list holds the previous round's ties only: in lockstep every
    // receiver hears the whole x plane, so a round without an R-phase tie
    // makes every receiver propose and then decide the majority (m > F, KIND 1
    // and 2 alike), and random starts tie with q(m) <= 10 % at m > 64.  So pass
    // r runs on grid >> 2(r - 1) workgroups: a full-size grid gives most waves
    // a single group, and every workgroup that works pays its serialised
    // deferral atomic and histogram flush (~12 ns each; N=256 F=0:
    // round 2 took 31 us for ~5 us of products).  The cooperative form's grid
    // is already one workgroup per group.
    const bool shrink = !benor::mfma_big_coop(kp);
    auto pass_grid = [&](uint32_t r) {
      if (!shrink || r < 2u) return grid;
      const int g = grid >> (2u * (r - 1u));
      return std::max(g, std::min(grid, 64));
    };
    // Deferral segments: a launch of u owners (waves, or workgroups of the
    // cooperative form) gives each at most ceil(groups / u) 32-trial groups,
    // so its segments hold that many trials each; the region is sized for the
    // largest u * cap over the chunk's launches (the per-launch cap is passed
    // in KParams::defer_seg_cap).
    const uint64_t groups = (cap + 31u) / 32u;
    auto seg_cap_of = [&](uint64_t units) { return (groups + units - 1u) / units * 32u; };
    uint64_t seg_words = 0;
    for (uint32_t r = 1u; r <= std::max<uint32_t>(last_round, 1u); ++r) {
      benor::KParams kr = kp;
      kr.cont_round = r >= 2u ? r : 0u;
      const uint64_t u = benor::defer_units(kr, pass_grid(r));
      seg_words = std::max<uint64_t>(seg_words, u * seg_cap_of(u));
    }
    const uint64_t words = 2u * cap + 64u + seg_words;                  // two lists, three lengths, segments
    // Test knob: a smaller segment capacity than the sizing rule's, so that a
    // GPU test can see the overflow reported (tests/test_mfma.py).
    const uint32_t test_seg_cap = benor::knob_u32("BENOR_TEST_DEFER_SEG_CAP", 0u);
    if (pl->defer_words < words) {
      if (pl->d_defer) (void)hipFree(pl->d_defer);
      pl->d_defer = nullptr;
      pl->defer_words = 0;
      HIP_TRY(hipMalloc(&pl->d_defer, sizeof(uint32_t) * words));
      pl->defer_words = words;
    }
    uint32_t *const lens = pl->d_defer + cap;                           // pass r's output length: lens[16 (r - 1)]
    uint32_t *const segs = lens + 64u;
    uint32_t *const lists[2] = {pl->d_defer, segs + seg_words};         // pass r writes lists[(r - 1) & 1]
    for (uint64_t done = 0; done < trial_count;) {
      const uint64_t n = std::min<uint64_t>(trial_count - done, cap);
      HIP_TRY(hipMemsetAsync(lens, 0, sizeof(uint32_t) * 16u * std::max<uint32_t>(last_round, 1u), s));   // every pass's length
      kp.trial_begin = trial_begin + done;
      kp.trial_count = n;
      kp.defer_seg = segs;
      uint32_t r_last = 1u;
      for (uint32_t r = 1u; r <= std::max<uint32_t>(last_round, 1u); ++r) {
        benor::KParams kc = kp;
        const int g = pass_grid(r);
        kc.cont_round = r >= 2u ? r : 0u;
        if (r >= 2u) {
          kc.trial_list = lists[(r - 2u) & 1u];
          kc.trial_list_len = lens + 16u * (r - 2u);
        }
        kc.defer_list = lists[(r - 1u) & 1u];
        kc.defer_len = lens + 16u * (r - 1u);
        kc.defer_seg_cap = (uint32_t)seg_cap_of(benor::defer_units(kc, g));
        if (test_seg_cap) kc.defer_seg_cap = std::min<uint32_t>(kc.defer_seg_cap, test_seg_cap);
        HIP_TRY(benor::launch_lockstep(kc, g, s));
        r_last = r;
      }
      benor::KParams kw = kp;
      kw.variant = kp.base_variant;              // W kernel (W <= 32) or blocked kernel
      kw.G = kp.base_G;
      kw.defer_list = kw.defer_len = kw.defer_seg = nullptr;
      kw.trial_list = lists[(r_last - 1u) & 1u];
      kw.trial_list_len = lens + 16u * (r_last - 1u);
      HIP_TRY(benor::launch_lockstep(kw, benor::lockstep_grid(kw, pl->device), s));
      done += n;
    }
    return BO_OK;
  }
  // Launches of at most 2^31 trials: the kernels index trials within a launch in 32 bits.
  for (uint64_t done = 0; done < trial_count;) {
    const uint64_t n = std::min<uint64_t>(trial_count - done, benor::kMaxTrialsPerLaunch);
    kp.trial_begin = trial_begin + done;
    kp.trial_count = n;
    const int grid = benor::lockstep_grid(kp, pl->device);
    const char *tl_path = kp.variant == 8 ? benor::knob("BENOR_TIMELINE") : nullptr;
    if (tl_path) {
      HIP_TRY(launch_with_timeline(kp, grid, s, tl_path));
    } else {
      HIP_TRY(benor::launch_lockstep(kp, grid, s));
    }
    done += n;
  }
  return BO_OK;
}

int bo_plan_launch(bo_plan *pl, uint64_t trial_begin, uint64_t trial_count, uint64_t *hist_dev, void *stream) {
  if (!pl || !hist_dev) return fail(BO_ERR_INVALID_ARGUMENT, "NULL argument");
  return plan_launch_impl(pl, trial_begin, trial_count, hist_dev, nullptr, nullptr,
                          reinterpret_cast<hipStream_t>(stream));
}

namespace {
int plan_flag_read(bo_plan *pl, hipStream_t s, uint32_t &v);
int plan_flag_error(uint32_t v);
}  // namespace

int bo_plan_run(bo_plan *pl, uint64_t trial_begin, uint64_t trial_count, uint64_t *hist_host) {
  if (!pl || !hist_host) return fail(BO_ERR_INVALID_ARGUMENT, "NULL argument");
  const uint32_t H = bo_hist_len(pl->cfg.k_max);
  uint64_t *d = nullptr;
  HIP_TRY(hipMalloc(&d, sizeof(uint64_t) * H));
  hipError_t e = hipMemset(d, 0, sizeof(uint64_t) * H);
  int rc = BO_OK;
  if (e == hipSuccess) rc = plan_launch_impl(pl, trial_begin, trial_count, d, nullptr, nullptr, nullptr);
  std::vector<uint64_t> h(H);
  if (e == hipSuccess && rc == BO_OK) e = hipMemcpy(h.data(), d, sizeof(uint64_t) * H, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(e, "bo_plan_run");
  if (rc) return rc;
  uint32_t flag = 0;
  rc = plan_flag_read(pl, nullptr, flag);   // the launches went to the null stream
  if (!rc) rc = plan_flag_error(flag);
  if (rc) return rc;
  for (uint32_t i = 0; i < H; ++i) hist_host[i] += h[i];
  return BO_OK;
}

namespace {
// The plan's invariant flag, read with a copy ordered on `s` (the stream its
// launches went to) on the plan's device: waits for that stream only, not for
// other plans', torch's or a live run's work (bo_plan_run, bo_consensus_wait).
// Cleared when set.
int plan_flag_read(bo_plan *pl, hipStream_t s, uint32_t &v) {
  v = 0;
  if (!pl->d_flag) return BO_OK;
  int cur = 0;
  HIP_TRY(hipGetDevice(&cur));
  if (cur != pl->device) HIP_TRY(hipSetDevice(pl->device));
  hipError_t e = hipMemcpyAsync(&v, pl->d_flag, sizeof v, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess && v) e = hipMemsetAsync(pl->d_flag, 0, sizeof v, s);
  if (e == hipSuccess && v) e = hipStreamSynchronize(s);
  if (cur != pl->device) (void)hipSetDevice(cur);
  if (e != hipSuccess) return hip_fail(e, "plan flag read");
  return BO_OK;
}

int plan_flag_error(uint32_t v) {
  if (!v) return BO_OK;
  if (v & 1u)
    return fail(BO_ERR_INTERNAL, "a matrix-core launch deferred more trials than its segment holds: "
                                 "its histogram is incomplete (deferral segment sizing)");
  return fail(BO_ERR_INTERNAL, "an event-level message pool filled up: the affected trials stopped early");
}
}  // namespace

// Standalone check after bo_plan_launch on streams the library does not know:
// the whole plan device is synchronised first.
int bo_plan_check(bo_plan *pl) {
  if (!pl) return fail(BO_ERR_INVALID_ARGUMENT, "NULL argument");
  if (!pl->d_flag) return BO_OK;
  int cur = 0;
  HIP_TRY(hipGetDevice(&cur));
  if (cur != pl->device) HIP_TRY(hipSetDevice(pl->device));
  const hipError_t e = hipDeviceSynchronize();
  if (cur != pl->device) (void)hipSetDevice(cur);
  if (e != hipSuccess) return hip_fail(e, "bo_plan_check");
  uint32_t v = 0;
  const int rc = plan_flag_read(pl, nullptr, v);
  return rc ? rc : plan_flag_error(v);
}

int bo_run_trials(const bo_trials_cfg *cfg, uint64_t trial_begin, uint64_t trial_count, uint64_t *hist_host) {
  bo_plan *pl = nullptr;
  int rc = bo_plan_create(cfg, &pl);
  if (rc) return rc;
  rc = bo_plan_run(pl, trial_begin, trial_count, hist_host);
  bo_plan_destroy(pl);
  return rc;
}

// One trial with per-node state in lockstep mode (the network API's
// /start, consensus.ts:3-8): every device operand -- live ids, initial planes,
// node states, histogram, round count -- goes into one per-thread device buffer
// that persists between calls, with one upload and one read-back.  A network of
// the reference's size is then a few tens of microseconds, not the ten
// allocations and frees of a plan.
namespace {
struct StateScratch {
  int device = -1;
  size_t bytes = 0;
  unsigned char *d = nullptr;
  std::vector<unsigned char> h;
  // no destructor: freeing device memory while the process exits can race the
  // HIP runtime's own teardown; the buffer is a few KB and the process owns it
};
thread_local StateScratch t_scratch;

int run_states_lockstep(const bo_trials_cfg *cfg, uint64_t trial, bo_node_state *nodes_out, uint32_t *rounds_out) {
  std::vector<uint32_t> live;
  std::vector<uint4> plane;
  benor::KParams kp;
  int rc = plan_host(cfg, live, plane, kp);
  if (rc) return rc;
  int dev = 0;
  rc = check_device(&dev);
  if (rc) return rc;
  const uint32_t N = cfg->N, H = bo_hist_len(cfg->k_max), m = kp.m;
  // layout: states [N] | hist [H] u64 | rounds u32 (+pad) | live [m] u32 | init [W] uint4
  const size_t o_st = 0, o_h = (sizeof(bo_node_state) * N + 15u) & ~size_t(15);
  const size_t o_r = o_h + sizeof(uint64_t) * H, o_live = (o_r + 16u + 15u) & ~size_t(15);
  const size_t o_init = (o_live + sizeof(uint32_t) * m + 15u) & ~size_t(15);
  const size_t bytes = o_init + sizeof(uint4) * plane.size();
  StateScratch &sc = t_scratch;
  if (sc.device != dev || sc.bytes < bytes) {
    if (sc.d) (void)hipFree(sc.d);
    sc.d = nullptr;
    sc.bytes = 0;
    HIP_TRY(hipMalloc(&sc.d, bytes));
    sc.bytes = bytes;
    sc.device = dev;
  }
  sc.h.assign(bytes, 0);
  // host-side initial states (node.ts:21-26); live entries are overwritten by the kernel
  bo_node_state *st = reinterpret_cast<bo_node_state *>(sc.h.data() + o_st);
  for (uint32_t i = 0; i < N; ++i) {
    const bool f = cfg->faulty[i] != 0;
    st[i].killed = f ? 1 : 0;
    st[i].x = f ? -1 : (cfg->init_mode == BO_INIT_FIXED ? cfg->init[i] : -1);
    st[i].decided = f ? -1 : 0;
    st[i].pad = 0;
    st[i].k = f ? -1 : 0;
  }
  if (m) std::memcpy(sc.h.data() + o_live, live.data(), sizeof(uint32_t) * m);
  if (!plane.empty()) std::memcpy(sc.h.data() + o_init, plane.data(), sizeof(uint4) * plane.size());
  HIP_TRY(hipMemcpy(sc.d, sc.h.data(), bytes, hipMemcpyHostToDevice));
  bo_plan pl;                      // on the stack: its device tables are views into the scratch buffer
  pl.kp = kp;
  pl.cfg = *cfg;
  pl.device = dev;
  pl.live_ids = live;
  pl.kp.live_ids = reinterpret_cast<uint32_t *>(sc.d + o_live);
  pl.kp.init_plane = reinterpret_cast<uint4 *>(sc.d + o_init);
  rc = plan_launch_impl(&pl, trial, 1, reinterpret_cast<uint64_t *>(sc.d + o_h),
                        reinterpret_cast<bo_node_state *>(sc.d + o_st), reinterpret_cast<uint32_t *>(sc.d + o_r),
                        nullptr);
  if (rc) return rc;
  HIP_TRY(hipMemcpy(sc.h.data(), sc.d, o_r + sizeof(uint32_t), hipMemcpyDeviceToHost));
  std::memcpy(nodes_out, sc.h.data() + o_st, sizeof(bo_node_state) * N);
  if (rounds_out) std::memcpy(rounds_out, sc.h.data() + o_r, sizeof(uint32_t));
  return BO_OK;
}
}  // namespace

namespace {
// Host-side initial states (node.ts:21-26); live entries are overwritten by the kernel.
void initial_states(const bo_trials_cfg *cfg, std::vector<bo_node_state> &st) {
  st.resize(cfg->N);
  for (uint32_t i = 0; i < cfg->N; ++i) {
    const bool f = cfg->faulty[i] != 0;
    st[i].killed = f ? 1 : 0;
    st[i].x = f ? -1 : (cfg->init_mode == BO_INIT_FIXED ? cfg->init[i] : -1);
    st[i].decided = f ? -1 : 0;
    st[i].pad = 0;
    st[i].k = f ? -1 : 0;
  }
}
}  // namespace

int bo_run_trial_states(const bo_trials_cfg *cfg, uint64_t trial, bo_node_state *nodes_out, uint32_t *rounds_out) {
  if (!cfg || !nodes_out) return fail(BO_ERR_INVALID_ARGUMENT, "NULL argument");
  if (cfg->mode == BO_MODE_LOCKSTEP) return run_states_lockstep(cfg, trial, nodes_out, rounds_out);
  bo_plan *pl = nullptr;
  int rc = bo_plan_create(cfg, &pl);
  if (rc) return rc;
  const uint32_t N = cfg->N, H = bo_hist_len(cfg->k_max);
  std::vector<bo_node_state> st;
  initial_states(cfg, st);
  bo_node_state *d_st = nullptr;
  uint64_t *d_h = nullptr;
  uint32_t *d_r = nullptr;
  hipError_t e = hipMalloc(&d_st, sizeof(bo_node_state) * N);
  if (e == hipSuccess) e = hipMalloc(&d_h, sizeof(uint64_t) * H);
  if (e == hipSuccess) e = hipMalloc(&d_r, sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemcpy(d_st, st.data(), sizeof(bo_node_state) * N, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(d_h, 0, sizeof(uint64_t) * H);
  if (e == hipSuccess) e = hipMemset(d_r, 0, sizeof(uint32_t));
  if (e == hipSuccess) rc = plan_launch_impl(pl, trial, 1, d_h, d_st, d_r, nullptr);
  uint32_t rounds = 0;
  if (e == hipSuccess && rc == BO_OK) e = hipMemcpy(nodes_out, d_st, sizeof(bo_node_state) * N, hipMemcpyDeviceToHost);
  if (e == hipSuccess && rc == BO_OK) e = hipMemcpy(&rounds, d_r, sizeof(uint32_t), hipMemcpyDeviceToHost);
  if (d_st) (void)hipFree(d_st);
  if (d_h) (void)hipFree(d_h);
  if (d_r) (void)hipFree(d_r);
  bo_plan_destroy(pl);
  if (e != hipSuccess) return hip_fail(e, "bo_run_trial_states");
  if (rc) return rc;
  if (rounds & 0x80000000u) return fail(BO_ERR_INTERNAL, "event-level message pool filled up: the run stopped early");
  if (rounds_out) *rounds_out = rounds;
  return BO_OK;
}

// ------------------------------------------------------------ live runs
namespace {
void slot_destroy(LiveSlot *sl) {
  if (sl->d) (void)hipFree(sl->d);
  if (sl->hp) (void)hipHostFree(sl->hp);
  if (sl->box) (void)hipHostFree(sl->box);
  if (sl->s) (void)hipStreamDestroy(sl->s);
  delete sl;
}

LiveSlot *slot_acquire(int dev) {
  {
    std::lock_guard<std::mutex> g(g_slots_mu);
    for (size_t i = 0; i < g_free_slots.size(); ++i)
      if (g_free_slots[i]->device == dev) {
        LiveSlot *sl = g_free_slots[i];
        g_free_slots.erase(g_free_slots.begin() + (long)i);
        return sl;
      }
  }
  auto *sl = new LiveSlot();
  sl->device = dev;
  const size_t box_bytes = sizeof(uint32_t) * benor::kLiveBoxWords;
  if (hipStreamCreateWithFlags(&sl->s, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void **>(&sl->box), box_bytes, hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void **>(&sl->dbox), sl->box, 0) != hipSuccess) {
    slot_destroy(sl);
    return nullptr;
  }
  return sl;
}

// Back to the pool after its run ended (the stream is idle): a large buffer is
// freed rather than kept (k concurrent N = 4096 runs kept k
// message pools of 268 MB for the life of the process).
void slot_release(LiveSlot *sl) {
  if (!sl) return;
  if (sl->bytes > kSlotKeepBytes) {
    (void)hipFree(sl->d);
    sl->d = nullptr;
    sl->bytes = 0;
  }
  std::lock_guard<std::mutex> g(g_slots_mu);
  g_free_slots.push_back(sl);
}

size_t align_up(size_t v, size_t a) { return (v + a - 1u) & ~(a - 1u); }

// One trial of a network on the workgroup-batched event kernel
// (benor_event_live.hip), on the slot's stream: the plan (host), the slot's
// buffer -- flag | states [N] | hist [H] | rounds | live ids [m] | init x [N]
// | stop schedule | message pool (HBM form only) -- one upload and the launch.
// `live`: the kernel polls the slot's mailbox for GET /stop and /getState.
int wg_launch(LiveSlot *sl, const bo_trials_cfg *cfg, bool live, WgRun &run) {
  std::vector<uint32_t> ids;
  std::vector<uint4> plane;
  benor::KParams kp;
  int rc = plan_host(cfg, ids, plane, kp, true);
  if (rc) return rc;
  const uint32_t N = cfg->N, H = bo_hist_len(cfg->k_max), m = kp.m;
  std::vector<uint64_t> stops;
  if (cfg->crash_at)
    for (uint32_t i = 0; i < N; ++i)
      if (cfg->crash_at[i] != 0xFFFFFFFFu) stops.push_back(((uint64_t)cfg->crash_at[i] << 12) | i);
  std::sort(stops.begin(), stops.end());
  const size_t o_st = 16u, o_h = align_up(o_st + sizeof(bo_node_state) * N, 16u);
  const size_t o_r = o_h + sizeof(uint64_t) * H, o_stats = align_up(o_r + 4u, 16u);
  const size_t o_live = o_stats + 24u * sizeof(uint64_t);
  const size_t o_ix = align_up(o_live + sizeof(uint32_t) * m, 16u);
  const size_t o_stops = align_up(o_ix + N, 16u);
  const size_t o_pool = align_up(o_stops + sizeof(uint64_t) * stops.size(), 256u);
  const size_t bytes = o_pool + (benor::event_wg_lds_pool(kp) ? 0u : (size_t)kp.ev_cap * 4u);
  if (sl->bytes < bytes) {
    if (sl->d) (void)hipFree(sl->d);
    sl->d = nullptr;
    sl->bytes = 0;
    HIP_TRY(hipMalloc(&sl->d, bytes));
    sl->bytes = bytes;
  }
  if (sl->hp_bytes < o_pool) {                  // (the slot's stream is idle: its last run ended)
    if (sl->hp) (void)hipHostFree(sl->hp);
    sl->hp = nullptr;
    sl->hp_bytes = 0;
    HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&sl->hp), o_pool, hipHostMallocDefault));
    sl->hp_bytes = o_pool;
  }
  unsigned char *const h = sl->hp;
  std::memset(h, 0, o_pool);
  std::vector<bo_node_state> st;
  initial_states(cfg, st);
  std::memcpy(h + o_st, st.data(), sizeof(bo_node_state) * N);
  if (m) std::memcpy(h + o_live, ids.data(), sizeof(uint32_t) * m);
  std::memcpy(h + o_ix, cfg->init, N);
  if (!stops.empty()) std::memcpy(h + o_stops, stops.data(), sizeof(uint64_t) * stops.size());
  if (live) {
    // the mailbox: no request, no stop landed, no snapshot asked (the slot's
    // previous kernel has ended)
    std::memset(sl->box, 0, sizeof(uint32_t) * benor::kLiveEv);
    for (uint32_t i = 0; i < N; ++i) sl->box[benor::kLiveEv + i] = 0xFFFFFFFFu;
    std::memset(sl->box + benor::kSnapReq, 0, sizeof(uint32_t) * (benor::kSnapSt - benor::kSnapReq));
  }
  HIP_TRY(hipMemcpyAsync(sl->d, h, o_pool, hipMemcpyHostToDevice, sl->s));
  kp.hist = reinterpret_cast<unsigned long long *>(sl->d + o_h);
  kp.overflow = reinterpret_cast<uint32_t *>(sl->d);
  kp.node_out = reinterpret_cast<bo_node_state *>(sl->d + o_st);
  kp.rounds_out = reinterpret_cast<uint32_t *>(sl->d + o_r);
  kp.live_ids = reinterpret_cast<uint32_t *>(sl->d + o_live);
  kp.init_x = reinterpret_cast<int8_t *>(sl->d + o_ix);
  kp.ev_stops = reinterpret_cast<uint64_t *>(sl->d + o_stops);
  kp.ev_nstops = (uint32_t)stops.size();
  kp.scratch = reinterpret_cast<uint32_t *>(sl->d + o_pool);
  kp.ev_lanes = 1u;                              // one trial
  kp.live_box = live ? sl->dbox : nullptr;
  kp.ev_stats = benor::knob("BENOR_EVENT_STATS") ? reinterpret_cast<unsigned long long *>(sl->d + o_stats) : nullptr;
  kp.trial_begin = 0;
  kp.trial_count = 1;
  run.o_st = o_st;
  run.o_r = o_r;
  run.o_stats = o_stats;
  run.N = N;
  run.F = cfg->F;
  HIP_TRY(benor::launch_event_wg(kp, 1, sl->s));
  HIP_TRY(hipMemcpyAsync(h, sl->d, o_r + 4u, hipMemcpyDeviceToHost, sl->s));   // read by wg_read
  return BO_OK;
}

// The run's head (flag | states | hist | rounds), read back on the slot's stream.
int wg_read(LiveSlot *sl, const WgRun &run, uint32_t N, std::vector<bo_node_state> &states) {
  if (const char *path = benor::knob("BENOR_EVENT_STATS")) {   // diagnostics: one JSON line per run
    unsigned long long s[24] = {};
    if (hipMemcpyAsync(s, sl->d + run.o_stats, sizeof s, hipMemcpyDeviceToHost, sl->s) == hipSuccess &&
        hipStreamSynchronize(sl->s) == hipSuccess)
      if (FILE *f = std::fopen(path, "a")) {
        static const char *names[23] = {"batches", "events", "batch_slots", "trigger_batches", "conflict_cut",
                                        "cyc_top", "cyc_picks", "cyc_lookup", "cyc_deliver", "cyc_cross",
                                        "cyc_writes_trigger", "cyc_bcast", "cycles", "wall_ticks", "cross_batches",
                                        "snapshots", "ev_work", "ev_wait", "ev_write", "ev_pre", "ev_drain",
                                        "cyc_trigger", "cyc_prepare"};
        std::fprintf(f, "{\"N\": %u, \"F\": %u", run.N, run.F);
        for (int i = 0; i < 23; ++i) std::fprintf(f, ", \"%s\": %llu", names[i], s[i]);
        std::fprintf(f, "}\n");
        std::fclose(f);
      }
  }
  // the head was copied into the pinned buffer behind the kernel (wg_launch)
  const hipError_t e = hipStreamSynchronize(sl->s);
  if (e != hipSuccess) return hip_fail(e, "event-level run");
  const unsigned char *head = sl->hp;
  uint32_t flag = 0, rounds = 0;
  std::memcpy(&flag, head, 4u);
  std::memcpy(&rounds, head + run.o_r, 4u);
  states.resize(N);
  std::memcpy(states.data(), head + run.o_st, sizeof(bo_node_state) * N);
  int rc = plan_flag_error(flag);
  if (!rc && (rounds & 0x80000000u))
    rc = fail(BO_ERR_INTERNAL, "event-level message pool filled up: the run stopped early");
  return rc;
}

// bo_consensus_start_sched with a /stop schedule: one trial on the
// workgroup-batched event kernel, synchronously.
int run_sched_wg(const bo_trials_cfg *cfg, std::vector<bo_node_state> &states) {
  int dev = 0;
  int rc = check_device(&dev);
  if (rc) return rc;
  LiveSlot *sl = slot_acquire(dev);
  if (!sl) return fail(BO_ERR_HIP, "event-level run: stream allocation failed");
  WgRun run;
  rc = wg_launch(sl, cfg, false, run);
  if (!rc) rc = wg_read(sl, run, cfg->N, states);
  if (hipStreamSynchronize(sl->s) == hipSuccess && rc != BO_ERR_HIP) slot_release(sl);
  else slot_destroy(sl);
  return rc;
}

// The end of a live run whose stream reported `e` (hipStreamSynchronize or a
// finished hipStreamQuery): read back, merge the final states, forget the run.
// Idempotent -- the first caller finalizes, later ones get its result.
int live_finalize(bo_network *net, const std::shared_ptr<bo_live> &lr, hipError_t e) {
  std::lock_guard<std::mutex> w(net->wait_mu);
  {
    std::lock_guard<std::mutex> g(net->mu);
    if (net->live != lr) return net->live_rc;
  }
  const uint32_t N = net->N;
  std::vector<bo_node_state> states;
  int rc = e != hipSuccess ? hip_fail(e, "bo_consensus_wait") : wg_read(lr->slot, lr->run, N, states);
  if (rc == BO_ERR_HIP) lr->failed = true;       // the slot's stream is not trusted again
  std::lock_guard<std::mutex> g(net->mu);
  net->live.reset();                             // from here a /stop is ordered after the run
  net->in_flight = false;
  net->live_rc = rc;
  if (!rc) {
    net->stop_events.assign(lr->slot->box + benor::kLiveEv, lr->slot->box + benor::kLiveEv + N);
    merge_states(net, lr->active, states);
  }
  return rc;
}
}  // namespace

bo_live::~bo_live() {
  if (!slot) return;
  if (failed || hipStreamSynchronize(slot->s) != hipSuccess) {
    // a faulted or aborted run: its stream, mailbox and buffer are not reused
    slot_destroy(slot);
  } else {
    slot_release(slot);
  }
}

// startConsensus whose GET /stop requests land while it runs (node.ts:191-194
// served during the round loop): the event-level kernel is launched and the
// call returns, as the reference's GET /start answers before consensus
// finishes (node.ts:167-188).  bo_node_stop / bo_consensus_stop post to the
// running kernel, bo_get_state(s) answer from its snapshots, and
// bo_consensus_wait / bo_consensus_poll end the run.
int bo_consensus_start_live(bo_network *net, uint64_t seed, uint32_t k_max) {
  StartPlan sp;
  int rc = start_prologue(net, k_max, nullptr, 0u, sp);
  if (rc || !sp.launch) return rc;
  const bo_trials_cfg cfg = start_cfg(net, seed, k_max, sp, BO_MODE_EVENT);
  int dev = 0;
  rc = check_device(&dev);
  auto lr = std::make_shared<bo_live>();
  lr->active = sp.active;
  if (!rc) {
    lr->slot = slot_acquire(dev);
    if (!lr->slot) rc = fail(BO_ERR_HIP, "live run: stream / mailbox allocation failed");
  }
  if (!rc) rc = wg_launch(lr->slot, &cfg, true, lr->run);
  std::lock_guard<std::mutex> g(net->mu);
  if (rc) {
    if (rc == BO_ERR_HIP) lr->failed = true;
    net->in_flight = false;
    net->started = false;          // nothing ran: the start may be retried
    return rc;
  }
  net->live = lr;
  net->live_rc = 0;
  net->stop_events.clear();
  // stops served between the prologue and now reach the kernel too
  std::vector<uint32_t> late;
  for (uint32_t i : sp.active)
    if (net->st[i].killed) late.push_back(i);
  if (!late.empty()) live_post(lr.get(), late.data(), (uint32_t)late.size());
  return BO_OK;
}

int bo_consensus_wait(bo_network *net) {
  if (!net) return fail(BO_ERR_INVALID_ARGUMENT, "net is NULL");
  std::shared_ptr<bo_live> lr;
  {
    std::lock_guard<std::mutex> g(net->mu);
    lr = net->live;
  }
  if (!lr) return BO_OK;
  const hipError_t e = hipStreamSynchronize(lr->slot->s);   // no lock held: /stop, /getState stay served
  return live_finalize(net, lr, e);
}

int bo_consensus_poll(bo_network *net, int *running_out) {
  if (!net || !running_out) return fail(BO_ERR_INVALID_ARGUMENT, "NULL argument");
  *running_out = 0;
  std::shared_ptr<bo_live> lr;
  {
    std::lock_guard<std::mutex> g(net->mu);
    lr = net->live;
  }
  if (!lr) return BO_OK;
  const hipError_t e = hipStreamQuery(lr->slot->s);
  if (e == hipErrorNotReady) {
    *running_out = 1;
    return BO_OK;
  }
  return live_finalize(net, lr, e);
}

namespace {
// Every node's state into out[N]: the network's own states, or -- while a live
// run is in flight -- a snapshot the kernel takes at its next batch boundary
// (the delivery count it reflects in *events_out), with the killed flags of
// GET /stop requests it has not applied yet (node.ts:191-194 sets killed at
// once).  A run that ends before it answers is finalized and its final states
// returned.
int get_states_impl(bo_network *net, bo_node_state *out, uint64_t *events_out) {
  if (events_out) *events_out = UINT64_MAX;
  std::shared_ptr<bo_live> lr;
  {
    std::lock_guard<std::mutex> g(net->mu);
    lr = net->live;
    if (!lr) {
      std::copy(net->st.begin(), net->st.end(), out);
      return net->live_rc;
    }
  }
  LiveSlot *sl = lr->slot;
  hipError_t q = hipStreamQuery(sl->s);
  if (q == hipErrorNotReady) {
    std::lock_guard<std::mutex> s(net->snap_mu);
    // a snapshot served within the last kSnapReuse answers this request too:
    // the reference's getNodesState is N concurrent GET /getState
    // (__test__/tests/utils.ts:14-20), and each snapshot costs the kernel its
    // host-memory writes (a tight poll loop slowed a run 4x)
    auto answer = [&]() {
      std::lock_guard<std::mutex> g(net->mu);
      std::copy(net->st.begin(), net->st.end(), out);   // nodes that do not run keep theirs
      for (size_t a = 0; a < lr->active.size(); ++a) {
        const uint32_t i = lr->active[a], w0 = lr->snap_words[2u * a], w1 = lr->snap_words[2u * a + 1u];
        bo_node_state s;
        s.killed = (int8_t)((w0 & 0xFFu) | (uint32_t)(net->st[i].killed != 0));   // /stop posted since
        s.x = (int8_t)(w0 >> 8);
        s.decided = (int8_t)(w0 >> 16);
        s.pad = 0;
        s.k = (int32_t)w1;
        out[i] = s;
      }
      if (events_out) *events_out = lr->snap_e;
      return BO_OK;
    };
    constexpr auto kSnapReuse = std::chrono::microseconds(500);
    if (lr->snap_ok && std::chrono::steady_clock::now() - lr->snap_t < kSnapReuse) return answer();
    uint32_t *box = sl->box;
    const uint32_t want = __atomic_add_fetch(&box[benor::kSnapReq], 1u, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
      if (__atomic_load_n(&box[benor::kSnapSeq], __ATOMIC_ACQUIRE) == want) {
        lr->snap_e = (uint64_t)__atomic_load_n(&box[benor::kSnapE], __ATOMIC_RELAXED) |
                     ((uint64_t)__atomic_load_n(&box[benor::kSnapE + 1u], __ATOMIC_RELAXED) << 32);
        lr->snap_words.resize(2u * lr->active.size());
        for (size_t a = 0; a < lr->active.size(); ++a) {
          const uint32_t i = lr->active[a];
          lr->snap_words[2u * a] = box[benor::kSnapSt + 2u * i];
          lr->snap_words[2u * a + 1u] = box[benor::kSnapSt + 2u * i + 1u];
        }
        lr->snap_t = std::chrono::steady_clock::now();
        lr->snap_ok = true;
        return answer();
      }
      if ((spin & 63u) == 63u) {
        q = hipStreamQuery(sl->s);
        if (q != hipErrorNotReady) break;          // the run ended before it served the request
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10))
          return fail(BO_ERR_INTERNAL, "a live run did not serve a /getState snapshot within 10 s");
        std::this_thread::yield();
      }
    }
  }
  const int rc = live_finalize(net, lr, q);
  std::lock_guard<std::mutex> g(net->mu);
  std::copy(net->st.begin(), net->st.end(), out);
  return rc;
}
}  // namespace

int bo_get_states(const bo_network *net, bo_node_state *out, uint32_t n, uint64_t *events_out) {
  if (!net || !out) return fail(BO_ERR_INVALID_ARGUMENT, "NULL argument");
  if (n != net->N) return fail(BO_ERR_INVALID_ARGUMENT, "out must have N entries");
  return get_states_impl(const_cast<bo_network *>(net), out, events_out);
}

int bo_live_stop_events(const bo_network *net, uint32_t *events_out, uint32_t n) {
  if (!net || !events_out) return fail(BO_ERR_INVALID_ARGUMENT, "NULL argument");
  if (n != net->N) return fail(BO_ERR_INVALID_ARGUMENT, "events_out must have N entries");
  std::lock_guard<std::mutex> g(net->mu);
  if (net->live) return fail(BO_ERR_INVALID_ARGUMENT, "a live run is in flight: bo_consensus_wait first");
  for (uint32_t i = 0; i < n; ++i) events_out[i] = i < net->stop_events.size() ? net->stop_events[i] : 0xFFFFFFFFu;
  return BO_OK;
}

double bo_popc_peak(uint32_t iters) {
  if (check_device(nullptr)) return 0.0;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  uint32_t *sink = nullptr;
  if (hipMalloc(&sink, sizeof(uint32_t) * cus * 8) != hipSuccess) return 0.0;
  const int grid = cus * 8, inner = 2048;
  double words = 0;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)benor::launch_popc_peak(sink, grid, inner, nullptr, &words);   // warm-up
  (void)hipEventRecord(a, nullptr);
  for (uint32_t i = 0; i < iters; ++i) (void)benor::launch_popc_peak(sink, grid, inner, nullptr, &words);
  (void)hipEventRecord(b, nullptr);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(sink);
  if (ms <= 0) return 0.0;
  return words * iters / (ms * 1e-3);
}

double bo_mfma_peak(uint32_t iters) {
  if (check_device(nullptr)) return 0.0;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  float *sink = nullptr;
  const int grid = cus * 2, inner = 4096;   // 2 waves per SIMD
  if (hipMalloc(&sink, sizeof(float) * grid) != hipSuccess) return 0.0;
  double terms = 0;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)benor::launch_mfma_peak(sink, grid, inner, nullptr, &terms);   // warm-up
  (void)hipEventRecord(a, nullptr);
  for (uint32_t i = 0; i < iters; ++i) (void)benor::launch_mfma_peak(sink, grid, inner, nullptr, &terms);
  (void)hipEventRecord(b, nullptr);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(sink);
  if (ms <= 0) return 0.0;
  return terms * iters / (ms * 1e-3);
}

}  // extern "C"
