"""A mid-run GET /stop through the reference's own API.

In the reference, startConsensus resolves as soon as every /start replied
(consensus.ts:5-7, node.ts:185-187), so a caller's GET /stop (node.ts:191-194)
lands while consensus runs, and from then on the stopped node drops every
message (node.ts:45).  Here a start carries that /stop as a schedule in
delivery counts (bo_consensus_start_sched; startConsensus(..., stop_after) in
Python, startConsensus(N, {stopAfter}) in js/index.js): the network API runs
the event-level kernel for one trial and serves its final per-node states.

GPU: per-node states equal oracle (iii) event_trial (oracle/benor_oracle.c,
trial 0 of the same seed and schedule) at N = 5, 10, 256, 1024 and 4096
(a network start with a schedule runs the live-run kernels of
benor_event_live.hip: registers at N <= 16, one wave at N <= 64, a workgroup
above), with stops inside round 1 and inside round 2, through the C ABI and
through the N-API addon.  CPU: the schedule's validation.
"""
import json
import os
import shutil
import subprocess

import pytest

import benor
import oracle
from conftest import ROOT

NEVER = None


def tied(m, n1):
    """m live initial values, n1 ones first."""
    return [1] * n1 + [0] * (m - n1)


def case(N, F, live_init, stops, seed, k_max=16):
    faulty = [i < F for i in range(N)]
    init = [0] * F + list(live_init)
    sched = [NEVER] * N
    for node, after in stops.items():
        sched[node] = after
    return {"N": N, "F": F, "faulty": faulty, "init": init, "stop_after": sched, "seed": seed, "k_max": k_max,
            "stops": stops}


def cases():
    """(case, round each scheduled stop must land in).  Round r of a trial
    with m running nodes spans deliveries [2 m N (r - 1), 2 m N r); tied
    starts (m even, as many 0s as 1s) make every node take its coin in round
    1, so the run reaches round 2.  Each landing round is checked on the
    oracle's states (the stopped node's k)."""
    out = []
    # N=5, F=1 (start.ts-sized, benorconsensus.test.ts shapes): m = 4, 40 deliveries per round
    out.append((case(5, 1, [1, 0, 1, 0], {2: 7}, seed=11), {2: 1}))
    out.append((case(5, 1, [1, 0, 1, 0], {3: 23}, seed=12), {3: 1}))
    out.append((case(5, 1, [1, 1, 0, 0], {1: 60}, seed=13), {1: 2}))
    # N=10, F=4 (test-suite shape): m = 6, 120 deliveries per round
    out.append((case(10, 4, tied(6, 3), {5: 30}, seed=21), {5: 1}))
    out.append((case(10, 4, tied(6, 3), {7: 150, 9: 190}, seed=22), {7: 2, 9: 2}))
    out.append((case(10, 4, [1, 1, 1, 1, 0, 1], {6: 60}, seed=23), {6: 1}))
    # N=256: F=85 (configs[2], m = 171 odd: decides in round 1, 87552 deliveries)
    out.append((case(256, 85, [(i * 7) % 3 == 0 and 1 or 0 for i in range(171)], {100: 1000, 200: 40000},
                     seed=31), {100: 1, 200: 1}))
    # N=256, F=84: m = 172, tied start, 88064 deliveries per round.  With exactly F
    # nodes faulty, a stopped live node leaves fewer than N - F senders: the run
    # stalls after it (node.ts:52, :88), as the reference's network hangs.
    out.append((case(256, 84, [i % 2 for i in range(172)], {90: 5000}, seed=32), {90: 1}))
    out.append((case(256, 84, [i % 2 for i in range(172)], {150: 140000}, seed=33), {150: 2}))
    out.extend(big_cases())
    return out


def big_cases():
    """Networks above the one-lane event kernel's N <= 256 (VERDICT r03 #2;
    the workgroup form of benor_event_live.hip since r06): BASELINE configs[3]'s N = 1024, F = 341 and configs[4]'s
    N = 4096, F = 1365.  m is odd there, so a random start decides in round 1;
    as many 1s as 0s plus one "?" make every R-phase tie (node.ts:63-69) and
    every node take its coin, so the run reaches round 2.  Round 1 spans
    2 m N deliveries (1 398 784 at N = 1024, 22 372 352 at N = 4096)."""
    def half(m):
        return [1] * (m // 2) + [0] * (m // 2) + ["?"]
    return [(case(1024, 341, half(683), {500: 300_000}, seed=41), {500: 1}),
            (case(1024, 341, half(683), {700: 1_900_000, 1000: 2_000_000}, seed=42), {700: 2, 1000: 2}),
            (case(4096, 1365, half(2731), {3000: 5_000_000}, seed=43), {3000: 1}),
            (case(4096, 1365, half(2731), {4000: 30_000_000}, seed=44), {4000: 2})]


def oracle_states(c):
    res, _ = oracle.event_trials(c["N"], c["F"], c["faulty"], seed=c["seed"], trial_begin=0, trial_count=1,
                                 k_max=c["k_max"], initial_values=c["init"], crash_at=c["stop_after"],
                                 want_states=True)
    st = res.states
    # the network API's auto-stop (node.ts:116-145): every node decided -> every node stopped
    if all(s["decided"] is True for s in st):
        st = [dict(s, killed=True) for s in st]
    return st


def test_schedule_validation():
    # a random /stop schedule (batch API crash_count) runs at every N since r05 (the
    # wave-per-trial kernel draws it per trial); planned on the host, no device needed
    for N in (300, 1024, 4096):
        assert benor.kernel_for(N, N // 3, [i < N // 3 for i in range(N)], mode=benor.BO_MODE_EVENT,
                                crash_count=3, crash_window=100) == benor.BO_KERNEL_EVENT
    benor.launchNetwork(5, 1, [1, 1, 1, 0, 0], [False, False, False, False, True])
    L = benor.lib()
    sched = (benor.ctypes.c_uint32 * 3)(1, 2, 3)
    assert L.bo_consensus_start_sched(benor._current._h, 1, 16, sched, 3) == benor.BO_ERR_INVALID_ARGUMENT
    # the mirrors refuse bad node ids and lengths before the C ABI sees them
    for bad in ({-1: 3}, {5: 3}, {"2": 3}, [1, 2, 3], {1: -4}, {1: 2.5}):
        with pytest.raises(ValueError):
            benor.startConsensus(5, seed=1, stop_after=bad)


def test_schedule_cases_land_where_intended():
    """The committed cases stop each node inside the round they name (oracle
    (iii) states: the stopped node is killed, at that k)."""
    for c, rounds in cases():
        st = oracle_states(c)
        for node, r in rounds.items():
            assert st[node]["killed"] and st[node]["k"] == r, (c["N"], c["F"], node, st[node])


@pytest.mark.gpu
@pytest.mark.parametrize("idx", range(len(cases())))
def test_network_api_stop_schedule_matches_oracle(idx):
    c, _ = cases()[idx]
    benor.launchNetwork(c["N"], c["F"], c["init"], c["faulty"])
    benor.startConsensus(c["N"], seed=c["seed"], k_max=c["k_max"], stop_after=c["stops"])
    assert benor.getNodesState(c["N"]) == oracle_states(c)
    for node in c["stops"]:
        assert benor.getStatus(node) == (500, "faulty")                 # node.ts:33-39 after the stop


@pytest.mark.gpu
def test_no_schedule_is_the_lockstep_start():
    """An all-NEVER schedule is bo_consensus_start (lockstep kernel), and the
    default start (event-level kernel, no stop sent) gives the same states."""
    c, _ = cases()[4]
    benor.launchNetwork(c["N"], c["F"], c["init"], c["faulty"])
    benor.startConsensus(c["N"], seed=c["seed"], k_max=c["k_max"], stop_after=[None] * c["N"])
    a = benor.getNodesState(c["N"])
    benor.launchNetwork(c["N"], c["F"], c["init"], c["faulty"])
    benor.startConsensus(c["N"], seed=c["seed"], k_max=c["k_max"])
    benor.waitConsensus(c["N"])
    assert benor.getNodesState(c["N"]) == a


SCRIPT = os.path.join(ROOT, "tests", "js", "stop_schedule.test.js")
ADDON = os.path.join(ROOT, "ben-or-consensus-algorithm_amd", "js", "benor.node")


@pytest.mark.gpu
@pytest.mark.skipif(shutil.which("node") is None or not os.path.exists(ADDON),
                    reason="node or the N-API addon is not available")
def test_js_stop_schedule_matches_oracle(tmp_path):
    """The same cases through js/index.js: launchNetwork -> startConsensus(N,
    {seed, kMax, stopAfter}) -> getNodesState."""
    payload = []
    for c, _ in cases():
        payload.append({k: c[k] for k in ("N", "F", "faulty", "init", "seed", "k_max")} |
                       {"stopAfter": {str(n): v for n, v in c["stops"].items()}, "expect": oracle_states(c)})
    f = tmp_path / "cases.json"
    f.write_text(json.dumps(payload))
    p = subprocess.run(["node", SCRIPT, str(f)], capture_output=True, text=True, timeout=120)
    print(p.stdout, p.stderr)
    assert p.returncode == 0, p.stdout + p.stderr
    assert f"{len(payload)} cases ok" in p.stdout
