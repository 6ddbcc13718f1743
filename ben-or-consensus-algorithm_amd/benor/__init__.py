"""Python mirror of the reference's public surface, over libbenor.so (C ABI).

The reference (viviendbk/ben-or-consensus-algorithm) exposes, in TypeScript:

    launchNetwork(N, F, initialValues, faultyList)   src/index.ts:4-14
    startConsensus(N) / stopConsensus(N)             src/nodes/consensus.ts:3-15
    GET /status, /getState on port 3000 + i          src/nodes/node.ts:33-39, :197-199
    getNodesState(N), reachedFinality(states)        __test__/tests/utils.ts:14-24

The same names, argument meanings and errors are provided here (the
JavaScript mirror for Node lives in ../js/).  As in the reference, one network
is "listening" at a time: startConsensus(N) / stopConsensus(N) / getNodesState(N)
address the network most recently launched.  Consensus itself runs as one HIP
kernel on the current device; there is no CPU fallback -- without the built
library or a gfx950 device every compute call raises.
"""
from __future__ import annotations

import ctypes
import os
import secrets
import struct
from typing import Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BENOR_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "lib", "libbenor.so")

BO_OK = 0
BO_ERR_ARRAYS_DONT_MATCH = 1
BO_ERR_FAULTY_COUNT = 2
BO_ERR_INVALID_ARGUMENT = 3
BO_ERR_NO_DEVICE = 4
BO_ERR_HIP = 5
BO_ERR_OUT_OF_RANGE = 6
BO_ERR_UNSUPPORTED = 7
BO_ERR_ALREADY_STARTED = 8
BO_MODE_LOCKSTEP = 0
BO_MODE_RANDOM_DELIVERY = 1
BO_MODE_EVENT = 2
NEVER = 0xFFFFFFFF             # crash_at entry: never stopped
BO_INIT_RANDOM = 0
BO_INIT_FIXED = 1
BO_KERNEL_NONE = -1
BO_KERNEL_BLOCKED = 0
BO_KERNEL_W = 1
BO_KERNEL_RANDOM = 2
BO_KERNEL_EVENT = 4
BO_KERNEL_LANE = 6
BO_KERNEL_MFMA = 7
BO_KERNEL_MFMA_SMALL = 8
KERNEL_NAMES = {BO_KERNEL_NONE: "none", BO_KERNEL_BLOCKED: "blocked popcount", BO_KERNEL_W: "W popcount",
                BO_KERNEL_RANDOM: "random delivery", BO_KERNEL_EVENT: "event level", BO_KERNEL_LANE: "lane",
                BO_KERNEL_MFMA: "matrix core (e2m1 MFMA)", BO_KERNEL_MFMA_SMALL: "packed matrix core (e2m1 MFMA, m <= 32)"}
BO_MAX_N = 4096
BO_MAX_K = 1024

# Environment knobs libbenor reads (csrc/benor_runtime.cpp kKnobs):
# none is needed in production; each forces a choice the planner makes itself.
# bench.py refuses to report while any is set.
KNOBS = {
    "BENOR_NO_MFMA": "validation", "BENOR_NO_MFMA_BIG": "validation", "BENOR_BIG_FORM": "validation",
    "BENOR_COOP_BW": "validation", "BENOR_SMALL_MIN_TRIALS": "validation", "BENOR_BLOCKS_PER_CU": "tuning",
    "BENOR_EVENT_LANES_PER_CU": "tuning", "BENOR_TEST_DEFER_SEG_CAP": "test", "BENOR_TIMELINE": "diagnostic",
    "BENOR_EVENT_FORM": "validation", "BENOR_LIVE_WAVES": "tuning", "BENOR_EVENT_STATS": "diagnostic",
}

BASE_NODE_PORT = 3000          # src/config.ts:1 (kept for the HTTP-shaped helpers)
DEFAULT_K_MAX = 64             # round cap; the reference runs until /stop

# Symbols the C ABI exports (include/benor.h); checked by tests.
EXPORTED_SYMBOLS = (
    "bo_network_create", "bo_consensus_start", "bo_consensus_stop", "bo_node_stop",
    "bo_get_state", "bo_status", "bo_network_size", "bo_network_destroy", "bo_hist_len",
    "bo_plan_create", "bo_plan_launch", "bo_plan_run", "bo_plan_popc_words_per_node_round",
    "bo_plan_live_nodes", "bo_plan_destroy", "bo_run_trials", "bo_run_trial_states",
    "bo_popc_peak", "bo_last_error", "bo_abi_version", "bo_kernel_version", "bo_plan_kernel", "bo_kernel_for",
    "bo_mfma_peak", "bo_consensus_start_sched", "bo_plan_check",
    "bo_consensus_start_live", "bo_consensus_wait", "bo_live_stop_events", "bo_get_states", "bo_consensus_poll",
)


class Error(Exception):
    """The reference's `new Error(message)` (launchNodes.ts:11,13)."""


class AlreadyStartedError(RuntimeError):
    """libbenor error 8: a second start on one network (its inboxes persist, node.ts:29-30)."""


class NodeStateC(ctypes.Structure):
    _fields_ = [("killed", ctypes.c_int8), ("x", ctypes.c_int8), ("decided", ctypes.c_int8),
                ("pad", ctypes.c_int8), ("k", ctypes.c_int32)]


class TrialsCfgC(ctypes.Structure):
    _fields_ = [("N", ctypes.c_uint32), ("F", ctypes.c_uint32), ("k_max", ctypes.c_uint32),
                ("init_mode", ctypes.c_uint32), ("mode", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("seed", ctypes.c_uint64), ("faulty", ctypes.POINTER(ctypes.c_uint8)),
                ("init", ctypes.POINTER(ctypes.c_int8)), ("crash_at", ctypes.POINTER(ctypes.c_uint32)),
                ("crash_count", ctypes.c_uint32), ("crash_window", ctypes.c_uint32)]


def _crash_array(N, crash_at):
    if crash_at is None:
        return None
    return (ctypes.c_uint32 * max(1, N))(*[NEVER if v is None else int(v) for v in crash_at])


_lib = None


def lib() -> ctypes.CDLL:
    """Load libbenor.so; raises if it was not built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libbenor.so not built at {LIB_PATH}: run __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    # int8 initial values and uint8 faulty flags, passed as bytes
    L.bo_network_create.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
                                    ctypes.c_char_p, ctypes.c_uint32, P(ctypes.c_void_p)]
    L.bo_consensus_start.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32]
    L.bo_consensus_start_sched.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, P(ctypes.c_uint32),
                                           ctypes.c_uint32]
    L.bo_consensus_start_live.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32]
    L.bo_consensus_wait.argtypes = [ctypes.c_void_p]
    L.bo_live_stop_events.argtypes = [ctypes.c_void_p, P(ctypes.c_uint32), ctypes.c_uint32]
    L.bo_consensus_stop.argtypes = [ctypes.c_void_p]
    L.bo_node_stop.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    L.bo_get_state.argtypes = [ctypes.c_void_p, ctypes.c_uint32, P(NodeStateC)]
    L.bo_get_states.argtypes = [ctypes.c_void_p, P(NodeStateC), ctypes.c_uint32, P(ctypes.c_uint64)]
    L.bo_consensus_poll.argtypes = [ctypes.c_void_p, P(ctypes.c_int)]
    L.bo_status.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    L.bo_network_size.argtypes = [ctypes.c_void_p]
    L.bo_network_size.restype = ctypes.c_uint32
    L.bo_network_destroy.argtypes = [ctypes.c_void_p]
    L.bo_network_destroy.restype = None
    L.bo_hist_len.argtypes = [ctypes.c_uint32]
    L.bo_hist_len.restype = ctypes.c_uint32
    L.bo_plan_create.argtypes = [P(TrialsCfgC), P(ctypes.c_void_p)]
    L.bo_plan_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                 ctypes.c_void_p]
    L.bo_plan_run.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, P(ctypes.c_uint64)]
    L.bo_plan_check.argtypes = [ctypes.c_void_p]
    L.bo_plan_popc_words_per_node_round.argtypes = [ctypes.c_void_p]
    L.bo_plan_popc_words_per_node_round.restype = ctypes.c_uint64
    L.bo_plan_live_nodes.argtypes = [ctypes.c_void_p]
    L.bo_plan_live_nodes.restype = ctypes.c_uint32
    L.bo_plan_destroy.argtypes = [ctypes.c_void_p]
    L.bo_plan_destroy.restype = None
    L.bo_run_trials.argtypes = [P(TrialsCfgC), ctypes.c_uint64, ctypes.c_uint64, P(ctypes.c_uint64)]
    L.bo_run_trial_states.argtypes = [P(TrialsCfgC), ctypes.c_uint64, P(NodeStateC), P(ctypes.c_uint32)]
    L.bo_popc_peak.argtypes = [ctypes.c_uint32]
    L.bo_popc_peak.restype = ctypes.c_double
    L.bo_mfma_peak.argtypes = [ctypes.c_uint32]
    L.bo_mfma_peak.restype = ctypes.c_double
    L.bo_plan_kernel.argtypes = [ctypes.c_void_p]
    L.bo_plan_kernel.restype = ctypes.c_int
    L.bo_kernel_for.argtypes = [P(TrialsCfgC), P(ctypes.c_int)]
    L.bo_last_error.restype = ctypes.c_char_p
    L.bo_abi_version.restype = ctypes.c_int
    L.bo_kernel_version.restype = ctypes.c_char_p
    _lib = L
    return L


def last_error() -> str:
    return lib().bo_last_error().decode()


def _check(rc: int) -> None:
    if rc != BO_OK:
        msg = last_error()
        if rc in (BO_ERR_ARRAYS_DONT_MATCH, BO_ERR_FAULTY_COUNT):
            raise Error(msg)
        if rc == BO_ERR_ALREADY_STARTED:
            raise AlreadyStartedError(f"libbenor error {rc}: {msg}")
        raise RuntimeError(f"libbenor error {rc}: {msg}")


_VAL = {0: 0, 1: 1, "?": 2}
_UNVAL = {-1: None, 0: 0, 1: 1, 2: "?"}


def _state_dict(s: NodeStateC) -> dict:
    """NodeState (src/types.ts:1-8)."""
    return {"killed": bool(s.killed), "x": _UNVAL[s.x],
            "decided": None if s.decided < 0 else bool(s.decided),
            "k": None if s.k < 0 else int(s.k)}


_REC = struct.Struct("bbbbi")                     # bo_node_state


def _state_dicts(arr, n: int) -> list[dict]:
    """n NodeState dicts from a bo_node_state array: a network's states repeat
    (a few distinct records at any N), so each distinct 8-byte record is
    decoded once and copied."""
    raw = memoryview(arr).cast("B").cast("Q")[:n]
    tab = {}
    for v in set(raw):
        kl, x, dec, _, k = _REC.unpack(v.to_bytes(8, "little"))
        tab[v] = {"killed": kl != 0, "x": _UNVAL[x], "decided": None if dec < 0 else dec != 0,
                  "k": None if k < 0 else k}
    return [tab[v].copy() for v in raw]


class Node:
    """Stands in for one of the `http.Server` objects launchNetwork returns:
    the caller may close() it (benorconsensus.test.ts:14-29); the node's
    routes are getState() / status()."""
    __slots__ = ("_net", "node_id")

    def __init__(self, net: "Network", node_id: int):
        self._net, self.node_id = net, node_id

    @property
    def port(self) -> int:
        return BASE_NODE_PORT + self.node_id

    def close(self, cb=None):
        if cb is not None:
            cb()

    def closeAllConnections(self):
        return None

    def getState(self) -> dict:
        return self._net.get_state(self.node_id)

    def status(self) -> tuple[int, str]:
        return self._net.status(self.node_id)


class Network:
    """Owns one bo_network handle (host-side node state)."""

    def __init__(self, N: int, F: int, initialValues: Sequence, faultyList: Sequence[bool]):
        L = lib()
        n_init, n_f = len(initialValues), len(faultyList)
        init = bytes(_VAL.get(v, -2) & 0xFF for v in initialValues) or b"\0"     # int8 values
        fl = bytes(v is True for v in faultyList) or b"\0"
        h = ctypes.c_void_p()
        _check(L.bo_network_create(N, F, init, n_init, fl, n_f, ctypes.byref(h)))
        self._h = h
        self.N, self.F = N, F

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.bo_network_destroy(h)
            self._h = None

    def start(self, seed: int | None = None, k_max: int = DEFAULT_K_MAX, stop_after=None) -> None:
        """stop_after: GET /stop requests that land during the run -- {node: deliveries} or a
        length-N sequence (None = not stopped); deliveries = POST /message handled network-wide
        before the stop (bo_consensus_start_sched: the event-level kernels, N <= 4096)."""
        if seed is None:
            seed = secrets.randbits(64)        # the reference's coin is Math.random()
        if not stop_after:
            _check(lib().bo_consensus_start(self._h, seed, k_max))
            return
        if not isinstance(stop_after, dict) and len(stop_after) != self.N:
            raise ValueError(f"stop_after: a sequence must have N = {self.N} entries, got {len(stop_after)}")
        sched = [None] * self.N
        for i, v in (stop_after.items() if isinstance(stop_after, dict) else enumerate(stop_after)):
            if isinstance(i, bool) or not isinstance(i, int) or not 0 <= i < self.N:
                raise ValueError(f"stop_after: node {i!r} is not a node id in [0, {self.N})")
            if v is not None and (isinstance(v, bool) or not isinstance(v, int) or not 0 <= v < NEVER):
                raise ValueError(f"stop_after[{i}]: {v!r} is not a delivery count (uint32 < 2^32 - 1) or None")
            sched[i] = v
        arr = _crash_array(self.N, sched)
        _check(lib().bo_consensus_start_sched(self._h, seed, k_max, arr, self.N))

    def start_live(self, seed: int | None = None, k_max: int = DEFAULT_K_MAX) -> None:
        """GET /start as the reference serves it (node.ts:167-188): launch the
        event-level kernel and return; stop() / stop_node() then land in the
        running kernel (bo_consensus_start_live) and wait() ends the run."""
        if seed is None:
            seed = secrets.randbits(64)
        _check(lib().bo_consensus_start_live(self._h, seed, k_max))

    def wait(self) -> None:
        """End of a live run: its final states replace the pre-run ones (no-op otherwise)."""
        _check(lib().bo_consensus_wait(self._h))

    def live_stop_events(self) -> list:
        """After wait(): per node, the delivery count at which the live run applied its
        /stop (None = none) -- as stop_after on a fresh network with the same seed it
        reproduces the run."""
        out = (ctypes.c_uint32 * max(1, self.N))()
        _check(lib().bo_live_stop_events(self._h, out, self.N))
        return [None if v == NEVER else int(v) for v in out[:self.N]]

    def stop(self) -> None:
        _check(lib().bo_consensus_stop(self._h))

    def stop_node(self, i: int) -> None:
        _check(lib().bo_node_stop(self._h, i))

    def poll(self) -> bool:
        """True while a live run is in flight; once it has ended its final states
        are merged (bo_consensus_poll, no blocking)."""
        r = ctypes.c_int(0)
        _check(lib().bo_consensus_poll(self._h, ctypes.byref(r)))
        return bool(r.value)

    def get_state(self, i: int) -> dict:
        """GET /getState (node.ts:197-199): at once, from a snapshot during a live run."""
        s = NodeStateC()
        _check(lib().bo_get_state(self._h, i, ctypes.byref(s)))
        return _state_dict(s)

    def get_states_at(self) -> tuple[list, int | None]:
        """Every node's state at once (bo_get_states) and, during a live run, the
        delivery count the snapshot reflects (None otherwise)."""
        st = (NodeStateC * max(1, self.N))()
        ev = ctypes.c_uint64(0)
        _check(lib().bo_get_states(self._h, st, self.N, ctypes.byref(ev)))
        return _state_dicts(st, self.N), (None if ev.value == 2 ** 64 - 1 else int(ev.value))

    def get_states(self) -> list[dict]:
        return self.get_states_at()[0]

    def status(self, i: int) -> tuple[int, str]:
        """GET /status (node.ts:33-39): (500, "faulty") or (200, "live")."""
        code = lib().bo_status(self._h, i)
        if code < 0:
            _check(-code)
        return (500, "faulty") if code == 500 else (200, "live")


_current: Network | None = None


def launchNetwork(N: int, F: int, initialValues: Sequence, faultyList: Sequence[bool]) -> list[Node]:
    """src/index.ts:4-14 -> launchNodes.ts:4-44.  Raises Error("Arrays don't
    match") / Error("faultyList doesnt have F faulties") like the reference."""
    global _current
    net = Network(N, F, initialValues, faultyList)
    _current = net
    return [Node(net, i) for i in range(N)]


def _net(N: int) -> Network:
    if _current is None or _current.N != N:
        raise RuntimeError(f"no launched network of size {N}")
    return _current


def startConsensus(N: int, seed: int | None = None, k_max: int = DEFAULT_K_MAX, stop_after=None,
                   strict: bool = False, live: bool | None = None, sync: bool = False) -> None:
    """src/nodes/consensus.ts:3-8: GET /start on every node.  As the
    reference's, it returns once the round loop (node.ts:43-163) is launched
    on the GPU, before consensus finishes (Network.start_live): stopConsensus /
    a node's stop land in the running kernel, getNodesState / getNodeState
    answer at once with the running network's states (a snapshot), and
    waitConsensus(N) waits for the end.  sync=True (or live=False) returns after the run (every live node
    decided, or k_max rounds; Network.start).  stop_after: a mid-run GET /stop
    schedule given up front (Network.start; returns after the run).  A second
    start on a network returns as the reference's does (every GET /start
    answers 200) but runs nothing: its inboxes persist (node.ts:29-30), so no
    fresh consensus can follow; strict=True raises instead."""
    if N == 0:
        return
    if live and stop_after:
        raise ValueError("stop_after and live are exclusive: a live run takes /stop as it comes")
    if live and sync:
        raise ValueError("live and sync are exclusive")
    if live is False:
        sync = True                      # an explicit non-live start is the run-to-completion form
    try:
        if not stop_after and not sync:
            _net(N).start_live(seed, k_max)
        else:
            _net(N).start(seed, k_max, stop_after)
    except AlreadyStartedError:
        if strict:
            raise


def stopConsensus(N: int) -> None:
    """src/nodes/consensus.ts:10-15: GET /stop on every node."""
    if N == 0:
        return
    _net(N).stop()


def getNodeState(nodeId: int) -> dict:
    """__test__/tests/utils.ts:4-12 (GET /getState, node.ts:197-199): answers at
    once -- during a live run, with the running network's state."""
    if _current is None:
        raise RuntimeError("no launched network")
    return _current.get_state(nodeId)


def getNodesState(N: int) -> list[dict]:
    """__test__/tests/utils.ts:14-20: every node's state at once (one snapshot of
    a running network, bo_get_states).  Callers poll it until reachedFinality, as
    the reference's tests do (benorconsensus.test.ts:153-160)."""
    return _net(N).get_states()


def waitConsensus(N: int) -> None:
    """The end of the network's live run (no-op otherwise): its final states."""
    if N == 0:
        return
    _net(N).wait()


def getStatus(nodeId: int) -> tuple[int, str]:
    if _current is None:
        raise RuntimeError("no launched network")
    return _current.status(nodeId)


def reachedFinality(states: Sequence[dict]) -> bool:
    """__test__/tests/utils.ts:22-24."""
    return all(s["decided"] is not False for s in states)


# ------------------------------------------------------------------ batches
def hist_len(k_max: int) -> int:
    return (k_max + 1) * 3 + 1


def _trials_cfg(N, F, faulty=None, *, seed=0, k_max=DEFAULT_K_MAX, initial_values=None, mode=BO_MODE_LOCKSTEP,
                crash_at=None, crash_count=0, crash_window=0):
    """bo_trials_cfg for a shape, and the ctypes arrays it points into."""
    if faulty is None:                       # start.ts:7-18 placement: the first F nodes
        faulty = [i < F for i in range(N)]
    fl = (ctypes.c_uint8 * max(1, N))(*[1 if v else 0 for v in faulty])
    if initial_values is None:
        init = (ctypes.c_int8 * max(1, N))()
        init_mode = BO_INIT_RANDOM
    else:
        init = (ctypes.c_int8 * max(1, N))(*[_VAL[v] for v in initial_values])
        init_mode = BO_INIT_FIXED
    crash = _crash_array(N, crash_at)
    cfg = TrialsCfgC(N, F, k_max, init_mode, mode, 0, seed,
                     ctypes.cast(fl, ctypes.POINTER(ctypes.c_uint8)),
                     ctypes.cast(init, ctypes.POINTER(ctypes.c_int8)),
                     ctypes.cast(crash, ctypes.POINTER(ctypes.c_uint32)) if crash else None,
                     crash_count, crash_window)
    return cfg, (fl, init, crash)


def kernel_for(N: int, F: int, faulty: Sequence[bool] | None = None, **kw) -> int:
    """The kernel family a TrialsPlan of this shape runs (bo_kernel_for; host only)."""
    cfg, _keep = _trials_cfg(N, F, faulty, **kw)
    k = ctypes.c_int()
    _check(lib().bo_kernel_for(ctypes.byref(cfg), ctypes.byref(k)))
    return k.value


class TrialsPlan:
    """Many independent trials of one (N, F, faulty) network shape on the
    current device (bo_plan_*)."""

    def __init__(self, N: int, F: int, faulty: Sequence[bool] | None = None, *, seed: int = 0,
                 k_max: int = DEFAULT_K_MAX, initial_values: Sequence | None = None,
                 mode: int = BO_MODE_LOCKSTEP, crash_at: Sequence | None = None, crash_count: int = 0,
                 crash_window: int = 0):
        self.N, self.F, self.k_max, self.seed = N, F, k_max, seed
        self.mode = mode
        self._cfg, self._keep = _trials_cfg(N, F, faulty, seed=seed, k_max=k_max, initial_values=initial_values,
                                            mode=mode, crash_at=crash_at, crash_count=crash_count,
                                            crash_window=crash_window)
        h = ctypes.c_void_p()
        _check(lib().bo_plan_create(ctypes.byref(self._cfg), ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.bo_plan_destroy(h)
            self._h = None

    @property
    def live_nodes(self) -> int:
        return lib().bo_plan_live_nodes(self._h)

    @property
    def popc_words_per_node_round(self) -> int:
        return lib().bo_plan_popc_words_per_node_round(self._h)

    @property
    def kernel(self) -> int:
        """BO_KERNEL_* family of this plan's batch launches (bo_plan_kernel)."""
        return lib().bo_plan_kernel(self._h)

    @property
    def hist_len(self) -> int:
        return hist_len(self.k_max)

    def launch(self, trial_begin: int, trial_count: int, hist_dev_ptr: int, stream_ptr: int = 0) -> None:
        """Asynchronous; adds into the device histogram at hist_dev_ptr."""
        _check(lib().bo_plan_launch(self._h, trial_begin, trial_count, ctypes.c_void_p(hist_dev_ptr),
                                    ctypes.c_void_p(stream_ptr)))

    def check(self) -> None:
        """bo_plan_check: synchronise and raise when a launch of this plan broke a
        device-side invariant (its histogram is then incomplete)."""
        _check(lib().bo_plan_check(self._h))

    def run(self, trial_begin: int, trial_count: int):
        import numpy as np

        h = np.zeros(self.hist_len, dtype=np.uint64)
        _check(lib().bo_plan_run(self._h, trial_begin, trial_count,
                                 h.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))
        return h


def run_trial_states(N: int, F: int, faulty: Sequence[bool], *, seed: int = 0, trial: int = 0,
                     k_max: int = DEFAULT_K_MAX, initial_values: Sequence | None = None,
                     mode: int = BO_MODE_LOCKSTEP, crash_at: Sequence | None = None, crash_count: int = 0,
                     crash_window: int = 0):
    """Per-node final states of one trial: (rounds, [NodeState dict] * N)."""
    fl = (ctypes.c_uint8 * max(1, N))(*[1 if v else 0 for v in faulty])
    if initial_values is None:
        init = (ctypes.c_int8 * max(1, N))()
        init_mode = BO_INIT_RANDOM
    else:
        init = (ctypes.c_int8 * max(1, N))(*[_VAL[v] for v in initial_values])
        init_mode = BO_INIT_FIXED
    ca = _crash_array(N, crash_at)
    cfg = TrialsCfgC(N, F, k_max, init_mode, mode, 0, seed,
                     ctypes.cast(fl, ctypes.POINTER(ctypes.c_uint8)),
                     ctypes.cast(init, ctypes.POINTER(ctypes.c_int8)),
                     ctypes.cast(ca, ctypes.POINTER(ctypes.c_uint32)) if ca else None, crash_count, crash_window)
    st = (NodeStateC * max(1, N))()
    rounds = ctypes.c_uint32(0)
    _check(lib().bo_run_trial_states(ctypes.byref(cfg), trial, st, ctypes.byref(rounds)))
    return int(rounds.value), [_state_dict(st[i]) for i in range(N)]


def kernel_version() -> str:
    """Digest of the kernel sources libbenor.so was built from."""
    return lib().bo_kernel_version().decode()


def popc_peak(iters: int = 20) -> float:
    return float(lib().bo_popc_peak(iters))


def mfma_peak(iters: int = 10) -> float:
    """Measured e2m1 32x32x64 MFMA multiply-adds per second (bo_mfma_peak)."""
    return float(lib().bo_mfma_peak(iters))
