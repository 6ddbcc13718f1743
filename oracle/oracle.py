"""ctypes front-end for the CPU oracle (oracle/benor_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.  It restates the
reference's algorithm (src/nodes/node.ts:43-163, launchNodes.ts:10-13); see the
C file header for the pinning story.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


class NodeState(ctypes.Structure):
    _fields_ = [("killed", ctypes.c_int8), ("x", ctypes.c_int8), ("decided", ctypes.c_int8),
                ("pad", ctypes.c_int8), ("k", ctypes.c_int32)]


class TrialsCfg(ctypes.Structure):
    _fields_ = [("N", ctypes.c_uint32), ("F", ctypes.c_uint32), ("k_max", ctypes.c_uint32),
                ("init_mode", ctypes.c_uint32), ("seed", ctypes.c_uint64),
                ("trial_begin", ctypes.c_uint64), ("trial_count", ctypes.c_uint64),
                ("faulty", ctypes.POINTER(ctypes.c_uint8)), ("init", ctypes.POINTER(ctypes.c_int8)),
                ("threads", ctypes.c_int32), ("mode", ctypes.c_uint32)]


def build() -> str:
    """Compile liboracle.so in place (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_philox4x32_10.argtypes = [ctypes.POINTER(ctypes.c_uint32)] * 3
        L.oracle_coin.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_coin.restype = ctypes.c_int
        L.oracle_random_init.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_random_init.restype = ctypes.c_int
        L.oracle_validate.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                      ctypes.POINTER(ctypes.c_uint8)]
        L.oracle_validate.restype = ctypes.c_int
        L.oracle_message_sim.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int8),
                                         ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(NodeState),
                                         ctypes.POINTER(ctypes.c_int)]
        L.oracle_message_sim.restype = ctypes.c_int
        L.oracle_run_trials.argtypes = [ctypes.POINTER(TrialsCfg), ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.POINTER(NodeState)]
        L.oracle_run_trials.restype = ctypes.c_int
        L.oracle_delivery_mask.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_delivery_mask.restype = None
        L.oracle_delivery_bernoulli.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                                ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_delivery_bernoulli.restype = ctypes.c_int
        L.oracle_event_trials.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.POINTER(NodeState), ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_event_trials.restype = ctypes.c_int
        L.oracle_event_states_at.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.POINTER(NodeState), ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_event_states_at.restype = ctypes.c_int
        _lib = L
    return _lib


def philox4x32_10(key, ctr):
    k = (ctypes.c_uint32 * 2)(*key)
    c = (ctypes.c_uint32 * 4)(*ctr)
    o = (ctypes.c_uint32 * 4)()
    lib().oracle_philox4x32_10(k, c, o)
    return list(o)


def coin(seed: int, trial: int, c: int, rnd: int) -> int:
    """Coin of the c-th live node (compact index) in round rnd >= 1."""
    return lib().oracle_coin(seed, trial, c, rnd)


def random_init(seed: int, trial: int, c: int, m: int) -> int:
    """Random initial value of the c-th live node of an m-live-node network
    (m <= 32: four consecutive trials share one Philox block)."""
    return lib().oracle_random_init(seed, trial, c, m)


VAL_CODE = {0: 0, 1: 1, "?": 2}
CODE_VAL = {-1: None, 0: 0, 1: 1, 2: "?"}


def _states(arr, n):
    out = []
    for i in range(n):
        s = arr[i]
        out.append({"killed": bool(s.killed), "x": CODE_VAL[s.x],
                    "decided": None if s.decided < 0 else bool(s.decided),
                    "k": None if s.k < 0 else int(s.k)})
    return out


def validate(N, F, initial_values, faulty_list) -> int:
    f = (ctypes.c_uint8 * max(1, len(faulty_list)))(*[1 if v else 0 for v in faulty_list])
    return lib().oracle_validate(N, F, len(initial_values), len(faulty_list), f)


def message_sim(N, F, initial_values, faulty_list, seed=0, trial=0, k_max=64, order_mode=1):
    """(i) message-level restatement: returns (rounds or -1, stalled, states)."""
    init = (ctypes.c_int8 * max(1, N))(*[VAL_CODE[v] for v in initial_values])
    f = (ctypes.c_uint8 * max(1, N))(*[1 if v else 0 for v in faulty_list])
    st = (NodeState * max(1, N))()
    stalled = ctypes.c_int(0)
    r = lib().oracle_message_sim(N, F, init, f, seed, trial, k_max, order_mode, st, ctypes.byref(stalled))
    return r, bool(stalled.value), _states(st, N)


def hist_len(k_max: int) -> int:
    return (k_max + 1) * 3 + 1


@dataclass
class TrialsResult:
    hist: np.ndarray
    states: list | None


def delivery_bernoulli(m: int, q: int):
    """(a, b) of the Bernoulli + fix-up sampler for (m, q), or None when the
    Floyd sampler is used."""
    a, b = ctypes.c_uint32(), ctypes.c_uint32()
    if lib().oracle_delivery_bernoulli(m, q, ctypes.byref(a), ctypes.byref(b)):
        return a.value, b.value
    return None


def delivery_mask(seed, trial, node, rnd, phase, m, q) -> list[int]:
    """Delivered-sender mask (list of W uint64 words) of one receiver-phase
    in the random-delivery model."""
    W = (m + 63) // 64
    D = (ctypes.c_uint64 * max(1, W))()
    lib().oracle_delivery_mask(seed, trial, node, rnd, phase, m, q, D)
    return [int(D[i]) for i in range(W)]


MODE_LOCKSTEP, MODE_RANDOM_DELIVERY, MODE_EVENT = 0, 1, 2


class EventCfg(ctypes.Structure):
    _fields_ = [("N", ctypes.c_uint32), ("F", ctypes.c_uint32), ("k_max", ctypes.c_uint32),
                ("init_mode", ctypes.c_uint32), ("seed", ctypes.c_uint64), ("trial_begin", ctypes.c_uint64),
                ("trial_count", ctypes.c_uint64), ("faulty", ctypes.POINTER(ctypes.c_uint8)),
                ("init", ctypes.POINTER(ctypes.c_int8)), ("crash_at", ctypes.POINTER(ctypes.c_uint32)),
                ("crash_count", ctypes.c_uint32), ("crash_window", ctypes.c_uint32), ("threads", ctypes.c_int32)]


NEVER = 0xFFFFFFFF


def event_trials(N, F, faulty_list, *, seed=0, trial_begin=0, trial_count=1, k_max=64, initial_values=None,
                 crash_at=None, crash_count=0, crash_window=0, threads=0, want_states=False):
    """(iii) event-level mode: message-granular run with seeded delivery order
    and scheduled (crash_at[i] = event index) or random mid-run /stop.
    Returns (TrialsResult, events delivered)."""
    f = (ctypes.c_uint8 * max(1, N))(*[1 if v else 0 for v in faulty_list])
    if initial_values is None:
        init, init_mode = (ctypes.c_int8 * max(1, N))(), 0
    else:
        init, init_mode = (ctypes.c_int8 * max(1, N))(*[VAL_CODE[v] for v in initial_values]), 1
    ca = None
    if crash_at is not None:
        ca = (ctypes.c_uint32 * max(1, N))(*[NEVER if v is None else int(v) for v in crash_at])
    cfg = EventCfg(N, F, k_max, init_mode, seed, trial_begin, trial_count,
                   ctypes.cast(f, ctypes.POINTER(ctypes.c_uint8)), ctypes.cast(init, ctypes.POINTER(ctypes.c_int8)),
                   ctypes.cast(ca, ctypes.POINTER(ctypes.c_uint32)) if ca is not None else None,
                   crash_count, crash_window, threads)
    hist = np.zeros(hist_len(k_max), dtype=np.uint64)
    st = (NodeState * max(1, N))() if want_states else None
    ev = ctypes.c_uint64(0)
    rc = lib().oracle_event_trials(ctypes.byref(cfg), hist.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), st,
                                   ctypes.byref(ev))
    if rc != 0:
        raise ValueError(f"oracle_event_trials rc={rc}")
    return TrialsResult(hist, _states(st, N) if want_states else None), int(ev.value)


def event_states_at(N, F, faulty_list, max_events, *, seed=0, trial=0, k_max=64, initial_values=None,
                    crash_at=None):
    """(iii) truncated before delivery `max_events` (after the stops scheduled
    there): the per-node states a live run's GET /getState snapshot taken at
    that delivery count must show (bo_get_states).  Returns (states, events
    delivered) -- fewer events when the run halted first."""
    f = (ctypes.c_uint8 * max(1, N))(*[1 if v else 0 for v in faulty_list])
    if initial_values is None:
        init, init_mode = (ctypes.c_int8 * max(1, N))(), 0
    else:
        init, init_mode = (ctypes.c_int8 * max(1, N))(*[VAL_CODE[v] for v in initial_values]), 1
    ca = None
    if crash_at is not None:
        ca = (ctypes.c_uint32 * max(1, N))(*[NEVER if v is None else int(v) for v in crash_at])
    cfg = EventCfg(N, F, k_max, init_mode, seed, 0, 1,
                   ctypes.cast(f, ctypes.POINTER(ctypes.c_uint8)), ctypes.cast(init, ctypes.POINTER(ctypes.c_int8)),
                   ctypes.cast(ca, ctypes.POINTER(ctypes.c_uint32)) if ca is not None else None, 0, 0, 1)
    st = (NodeState * max(1, N))()
    ev = ctypes.c_uint64(0)
    rc = lib().oracle_event_states_at(ctypes.byref(cfg), trial, max_events, st, ctypes.byref(ev))
    if rc != 0:
        raise ValueError(f"oracle_event_states_at rc={rc}")
    return _states(st, N), int(ev.value)


def run_trials(N, F, faulty_list, *, seed=0, trial_begin=0, trial_count=1, k_max=64,
               initial_values=None, threads=0, want_states=False, mode=MODE_LOCKSTEP) -> TrialsResult:
    """(ii) round-level bit-plane restatement over a batch of trials."""
    f = (ctypes.c_uint8 * max(1, N))(*[1 if v else 0 for v in faulty_list])
    if initial_values is None:
        init = (ctypes.c_int8 * max(1, N))()
        init_mode = 0
    else:
        init = (ctypes.c_int8 * max(1, N))(*[VAL_CODE[v] for v in initial_values])
        init_mode = 1
    cfg = TrialsCfg(N, F, k_max, init_mode, seed, trial_begin, trial_count,
                    ctypes.cast(f, ctypes.POINTER(ctypes.c_uint8)),
                    ctypes.cast(init, ctypes.POINTER(ctypes.c_int8)), threads, mode)
    hist = np.zeros(hist_len(k_max), dtype=np.uint64)
    st = (NodeState * max(1, N))() if want_states else None
    rc = lib().oracle_run_trials(ctypes.byref(cfg), hist.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                 st)
    if rc != 0:
        raise ValueError(f"oracle_run_trials rc={rc}")
    return TrialsResult(hist, _states(st, N) if want_states else None)
