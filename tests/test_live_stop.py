"""GET /stop served while consensus runs, as the reference serves it (VERDICT r03
"missing" #2: ad-hoc /stop ordering).

In the reference, startConsensus resolves once every GET /start replied
(consensus.ts:5-7, node.ts:185-187); a GET /stop (node.ts:191-194) that the
caller sends afterwards lands wherever the round loop happens to be, and the
stopped node drops every later message (node.ts:45).  bo_consensus_start_live
runs the event-level kernel on its own stream and returns; bo_node_stop /
bo_consensus_stop post to a host-mapped mailbox the kernel polls, each request
lands before the next delivery, and that delivery count comes back
(bo_live_stop_events).  Where a request lands depends on wall-clock timing, so
the parity check is a replay: the recorded counts as a stop schedule through
oracle (iii) event_trial (oracle/benor_oracle.c, trial 0 of the same seed) and
through bo_consensus_start_sched must give the live run's states exactly.

CPU: argument checks and the no-device path.  GPU: live runs at N = 10,
1024 and 4096 against the oracle, with stops posted at once, after a delay,
after the run, and to every node; the same through js/index.js.
"""
import json
import os
import shutil
import subprocess
import time

import pytest

import benor
import oracle
from conftest import ROOT


def half(m):
    """m live values (m odd): as many 1s as 0s plus one "?" -- every R-phase
    ties (node.ts:63-69), every node takes its coin, the run reaches round 2."""
    return [1] * (m // 2) + [0] * (m // 2) + ["?"]


def shape(N, F, live_init):
    return [i < F for i in range(N)], [0] * F + list(live_init)


def expected(N, F, faulty, init, seed, k_max, stop_after):
    res, _ = oracle.event_trials(N, F, faulty, seed=seed, trial_begin=0, trial_count=1, k_max=k_max,
                                 initial_values=init, crash_at=stop_after, want_states=True)
    st = res.states
    if all(s["decided"] is True for s in st):         # the network API's auto-stop (node.ts:116-145)
        st = [dict(s, killed=True) for s in st]
    return st


def expected_live(N, F, faulty, init, seed, k_max, events, requested):
    """The states of a live run whose /stop requests landed at `events`; a
    requested node whose request came after the run ended (event None) keeps
    its final state and is killed."""
    st = expected(N, F, faulty, init, seed, k_max, events)
    return [dict(s, killed=True) if i in requested and events[i] is None else s for i, s in enumerate(st)]


def test_live_api_checks():
    faulty, init = shape(10, 4, [1, 0, 1, 0, 1, 0])
    net = benor.Network(10, 4, init, faulty)
    net.wait()                                         # nothing in flight: a no-op
    assert net.live_stop_events() == [None] * 10       # no live run yet
    L = benor.lib()
    out = (benor.ctypes.c_uint32 * 3)()
    assert L.bo_live_stop_events(net._h, out, 3) == benor.BO_ERR_INVALID_ARGUMENT
    benor.launchNetwork(10, 4, init, faulty)
    with pytest.raises(ValueError):
        benor.startConsensus(10, seed=1, live=True, stop_after={5: 3})


def test_live_start_without_device_can_be_retried():
    """No gfx950 device: the start fails loudly (no CPU fallback) and the network
    stays unstarted.  On a GPU box this is a plain live run."""
    faulty, init = shape(10, 4, [1, 0, 1, 0, 1, 0])
    net = benor.Network(10, 4, init, faulty)
    try:
        net.start_live(seed=3, k_max=16)
    except RuntimeError as e:
        assert "libbenor error 4" in str(e)
        with pytest.raises(RuntimeError, match="libbenor error 4"):
            net.start_live(seed=3, k_max=16)           # not error 8: nothing ran
        return
    net.wait()
    assert net.get_state(4)["k"] >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("N,F", [(10, 4), (1024, 341)])
def test_live_run_without_stops_matches_oracle(N, F):
    faulty, init = shape(N, F, half(N - F) if (N - F) % 2 else [1, 0] * ((N - F) // 2))
    net = benor.Network(N, F, init, faulty)
    net.start_live(seed=61, k_max=16)
    net.wait()
    assert net.live_stop_events() == [None] * N
    assert [net.get_state(i) for i in range(N)] == expected(N, F, faulty, init, 61, 16, None)


@pytest.mark.gpu
def test_live_stops_land_mid_run_and_replay():
    """N = 1024, F = 341 (configs[3]): one /stop posted at once, one 20 ms later
    (a round is ~1.4 M deliveries here).  The first lands in the run, the second
    lands or is ordered after it; the recorded delivery counts replayed as a
    schedule -- through the oracle and through bo_consensus_start_sched on a
    fresh network -- give the same states."""
    N, F, seed = 1024, 341, 62
    faulty, init = shape(N, F, half(N - F))
    net = benor.Network(N, F, init, faulty)
    net.start_live(seed=seed, k_max=16)
    net.stop_node(500)
    assert net.status(500) == (500, "faulty")         # GET /status answers at once
    time.sleep(0.02)
    net.stop_node(900)
    net.wait()
    ev = net.live_stop_events()
    # the first request is posted microseconds after the launch, long before the
    # run can end; the second may come after it (the stop of node 500 leaves
    # fewer than N - F senders, so the run drains its pool and stalls)
    assert ev[500] is not None, ev[500]
    assert ev[900] is None or ev[500] <= ev[900]
    assert sum(v is not None for v in ev) == 1 + (ev[900] is not None)
    states = [net.get_state(i) for i in range(N)]
    assert states[500]["killed"] and states[900]["killed"]
    assert states == expected_live(N, F, faulty, init, seed, 16, ev, {500, 900})
    replay = benor.Network(N, F, init, faulty)
    replay.start(seed=seed, k_max=16, stop_after=ev)
    if ev[900] is None:
        replay.stop_node(900)
    assert [replay.get_state(i) for i in range(N)] == states


@pytest.mark.gpu
def test_live_stop_consensus_at_4096():
    """N = 4096, F = 1365 (configs[4]): stopConsensus right after the start
    stops every running node within the first poll interval; one delivery
    count for all of them, and the replay agrees."""
    N, F, seed = 4096, 1365, 63
    faulty, init = shape(N, F, half(N - F))
    net = benor.Network(N, F, init, faulty)
    net.start_live(seed=seed, k_max=16)
    time.sleep(0.01)
    net.stop()
    net.wait()
    ev = net.live_stop_events()
    landed = {v for i, v in enumerate(ev) if not faulty[i]}
    assert len(landed) == 1 and None not in landed, sorted(landed, key=str)[:4]
    assert all(ev[i] is None for i in range(F))       # faulty nodes never ran
    states = [net.get_state(i) for i in range(N)]
    assert all(s["killed"] for s in states)
    assert states == expected(N, F, faulty, init, seed, 16, ev)


@pytest.mark.gpu
def test_live_stop_after_the_run_is_ordered_after_it():
    """N = 10: the run ends in microseconds; a /stop served after wait() keeps
    the node's final x / decided / k and kills it, as for a synchronous start."""
    N, F, seed = 10, 4, 64
    faulty, init = shape(N, F, [1, 0, 1, 0, 1, 0])
    net = benor.Network(N, F, init, faulty)
    net.start_live(seed=seed, k_max=16)
    net.wait()
    net.stop_node(6)
    ref = expected(N, F, faulty, init, seed, 16, None)
    got = [net.get_state(i) for i in range(N)]
    assert got[6] == dict(ref[6], killed=True)
    assert got[:6] + got[7:] == ref[:6] + ref[7:]
    assert net.live_stop_events() == [None] * N


@pytest.mark.gpu
def test_module_api_live_start_then_wait():
    """benor.startConsensus(N, live=True) returns before the run ends;
    getNodesState(N) answers at once (a snapshot, checked in
    test_live_snapshots_*), waitConsensus(N) gives the final states."""
    N, F, seed = 1024, 341, 65
    faulty, init = shape(N, F, half(N - F))
    benor.launchNetwork(N, F, init, faulty)
    benor.startConsensus(N, seed=seed, k_max=16, live=True)
    assert len(benor.getNodesState(N)) == N
    benor.waitConsensus(N)
    assert benor.getNodesState(N) == expected(N, F, faulty, init, seed, 16, None)


@pytest.mark.gpu
@pytest.mark.parametrize("N,F,seed", [(10, 4, 81), (1024, 341, 82)])
def test_default_start_then_stop_consensus_replays(N, F, seed):
    """the reference's call sequence -- startConsensus(N) with
    no option, then stopConsensus(N) at once (consensus.ts:3-15) -- lands the
    stops in the running kernel.  The per-node states equal oracle (iii)'s
    replay of the recorded delivery counts.  At N = 1024 the run lasts
    milliseconds, so the stops must land in it; at N = 10 a run of ~100
    deliveries can end before the request reaches the kernel, and a stop it
    did not see is ordered after the run (the replay covers both)."""
    faulty, init = shape(N, F, half(N - F) if (N - F) % 2 else [1, 0] * ((N - F) // 2))
    benor.launchNetwork(N, F, init, faulty)
    benor.startConsensus(N, seed=seed, k_max=16)
    benor.stopConsensus(N)
    benor.waitConsensus(N)
    states = benor.getNodesState(N)
    ev = benor._current.live_stop_events()
    running = set(range(F, N))
    if N >= 1024:
        assert all(ev[i] is not None for i in running), [ev[i] for i in range(F, F + 4)]
        assert len({ev[i] for i in running}) == 1       # one request for every node, one landing point
    assert all(ev[i] is None for i in range(F))       # faulty nodes never ran
    assert all(s["killed"] for s in states)
    assert states == expected_live(N, F, faulty, init, seed, 16, ev, set(range(N)))


@pytest.mark.gpu
@pytest.mark.parametrize("N,F", [(78, 26), (79, 26)])
def test_live_pool_in_lds_and_in_hbm_replay(N, F):
    """The two forms of a live run: at N = 78 the message pool (4N^2 + 64
    words) fits kEventBigLdsPool and lives in LDS; at N = 79 it is in HBM
    (benor_event_live.hip; the control wave polls the mailbox either way).  A stop
    for a third of the running nodes sent right after the default start; the
    states equal oracle (iii)'s replay of the recorded landing points."""
    seed = 0x4C50 + N
    faulty, init = shape(N, F, half(N - F) if (N - F) % 2 else [1, 0] * ((N - F) // 2))
    benor.launchNetwork(N, F, init, faulty)
    benor.startConsensus(N, seed=seed, k_max=16)
    stopped = set(range(F, N, 3))
    for i in sorted(stopped):
        benor._current.stop_node(i)                 # GET /stop on node i (node.ts:191-194)
    benor.waitConsensus(N)
    states = benor.getNodesState(N)
    ev = benor._current.live_stop_events()
    assert all(ev[i] is None for i in range(F))
    assert all(states[i]["killed"] for i in stopped)
    assert states == expected_live(N, F, faulty, init, seed, 16, ev, stopped)


SCRIPT = os.path.join(ROOT, "tests", "js", "live_stop.test.js")
ADDON = os.path.join(ROOT, "ben-or-consensus-algorithm_amd", "js", "benor.node")


@pytest.mark.gpu
@pytest.mark.skipif(shutil.which("node") is None or not os.path.exists(ADDON),
                    reason="node or the N-API addon is not available")
def test_js_live_stop_replays_through_oracle(tmp_path):
    """js/index.js: startConsensus(N, {live: true}) -> stopNode -> getNodesState,
    liveStopEvents; the states must be the oracle's for the recorded counts."""
    cases = []
    for N, F, seed, stops in ((10, 4, 71, [5]), (1024, 341, 72, [400, 800])):
        faulty, init = shape(N, F, half(N - F) if (N - F) % 2 else [1, 0] * ((N - F) // 2))
        cases.append({"N": N, "F": F, "faulty": faulty, "init": init, "seed": seed, "stops": stops})
    f = tmp_path / "cases.json"
    f.write_text(json.dumps(cases))
    out = tmp_path / "out.json"
    p = subprocess.run(["node", SCRIPT, str(f), str(out)], capture_output=True, text=True, timeout=120)
    print(p.stdout, p.stderr)
    assert p.returncode == 0, p.stdout + p.stderr
    results = json.loads(out.read_text())
    assert len(results) == len(cases)
    for c, r in zip(cases, results):
        ev = r["events"]
        assert len(ev) == c["N"]
        assert r["states"] == expected_live(c["N"], c["F"], c["faulty"], c["init"], c["seed"], 16, ev,
                                            set(c["stops"]))
        for i in c["stops"]:
            assert r["states"][i]["killed"]


@pytest.mark.gpu
def test_live_edge_cases():
    """A one-node network; a /stop posted twice and to a faulty node (both
    no-ops beyond the first); a network dropped while its live run is in flight
    (destroy waits for it); a second live start (refused, error 8)."""
    # N = 1: the lone node decides its own value in round 1, all decided -> auto-stop
    net = benor.Network(1, 0, [1], [False])
    net.start_live(seed=1, k_max=16)
    net.wait()
    assert net.get_state(0) == {"killed": True, "x": 1, "decided": True, "k": 2}
    # repeated and faulty-node stops
    N, F, seed = 1024, 341, 66
    faulty, init = shape(N, F, half(N - F))
    net = benor.Network(N, F, init, faulty)
    net.start_live(seed=seed, k_max=16)
    net.stop_node(700)
    net.stop_node(700)
    net.stop_node(3)                                  # faulty from launch: already killed
    with pytest.raises(benor.AlreadyStartedError):
        net.start_live(seed=seed, k_max=16)
    net.wait()
    ev = net.live_stop_events()
    assert ev[3] is None and sum(v is not None for v in ev) == (ev[700] is not None)
    assert [net.get_state(i) for i in range(N)] == expected_live(N, F, faulty, init, seed, 16, ev, {3, 700})
    # dropped mid-run: the handle's destructor waits for the kernel
    other = benor.Network(N, F, init, faulty)
    other.start_live(seed=seed + 1, k_max=16)
    del other
