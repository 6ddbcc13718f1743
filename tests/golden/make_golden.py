"""Generate the committed golden fixtures under tests/golden/.

reference_cases.json
    The reference's own known-answer tests, as data: inputs and the assertions
    __test__/tests/benorconsensus.test.ts makes on them (line ranges cited per
    case), plus the launch-validation errors of src/nodes/launchNodes.ts:10-13.
    These pin the oracle (tests/test_oracle.py) -- the reference itself cannot
    run in this image.

oracle_vectors.json
    Seeded per-node final states and outcome histograms produced by the CPU
    oracle (oracle/benor_oracle.c), with the message-level restatement (i)
    and the bit-plane restatement (ii) required to agree before anything is
    written.  The GPU parity tests compare the HIP kernel against these.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import itertools
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402

T, F_ = True, False
TEST = "__test__/tests/benorconsensus.test.ts"

REFERENCE_CASES = [
    {"name": "Can start 2 healthy nodes and 1 faulty node", "src": f"{TEST}:45-75",
     "N": 3, "faulty": [T, F_, F_], "init": [1, 1, 1], "start": False,
     "expect": {"status": [[500, "faulty"], [200, "live"], [200, "live"]]}},
    {"name": "Can start 8 healthy nodes and 2 faulty nodes", "src": f"{TEST}:77-118",
     "N": 10, "faulty": [T, F_, F_, F_, F_, T, F_, F_, F_, F_], "init": [1] * 10, "start": False,
     "expect": {"status": [[500, "faulty"] if f else [200, "live"] for f in
                           [T, F_, F_, F_, F_, T, F_, F_, F_, F_]]}},
    {"name": "Finality is reached - Unanimous Agreement", "src": f"{TEST}:133-175",
     "N": 5, "faulty": [F_] * 5, "init": [1] * 5, "start": True,
     "expect": {"faulty_null": True, "live": {"decided": "truthy", "x": 1, "k_le": 2}}},
    {"name": "Finality is reached - Simple Majority", "src": f"{TEST}:179-223",
     "N": 5, "faulty": [F_, F_, F_, F_, T], "init": [1, 1, 1, 0, 0], "start": True,
     "expect": {"faulty_null": True, "live": {"decided": "truthy", "x": 1, "k_le": 2}}},
    {"name": "Finality is reached - Fault Tolerance Threshold", "src": f"{TEST}:227-286",
     "N": 9, "faulty": [T, T, T, T, F_, F_, F_, F_, F_], "init": [0, 0, 1, 1, 1, 0, 0, 1, 1], "start": True,
     "expect": {"faulty_null": True, "live": {"decided": "truthy", "k": "not_null", "x": "not_null"},
                "agreement": True}},
    {"name": "Finality is reached - Exceeding Fault Tolerance", "src": f"{TEST}:292-345",
     "N": 10, "faulty": [T] * 5 + [F_] * 5, "init": [0, 0, 1, 1, 1, 0, 0, 1, 1, 0], "start": True,
     "expect": {"faulty_null": True, "live": {"decided": "falsy", "k_gt": 10, "x": "not_null"}}},
    {"name": "Finality is reached - No Faulty Nodes", "src": f"{TEST}:351-393",
     "N": 5, "faulty": [F_] * 5, "init": [0, 1, 0, 1, 1], "start": True,
     "expect": {"faulty_null": True, "live": {"decided": "truthy", "x": 1, "k_le": 2}}},
    {"name": "Finality is reached - Randomized", "src": f"{TEST}:399-450",
     "N": 7, "faulty": [F_, F_, T, F_, T, F_, F_], "init": "random01", "start": True,
     "expect": {"faulty_null": True, "live": {"decided": "truthy", "x": "not_null"}, "agreement": True}},
    {"name": "Hidden Test - Finality is reached - One node", "src": f"{TEST}:454-486",
     "N": 1, "faulty": [F_], "init": [1], "start": True,
     "expect": {"length": 1, "live": {"decided": "truthy", "x": 1}}},
]

LAUNCH_ERRORS = [
    {"src": "src/nodes/launchNodes.ts:10-11", "N": 3, "F": 0, "init": [1, 1], "faulty": [F_, F_, F_],
     "error": "Arrays don't match"},
    {"src": "src/nodes/launchNodes.ts:10-11", "N": 4, "F": 0, "init": [1, 1, 1], "faulty": [F_, F_, F_],
     "error": "Arrays don't match"},
    {"src": "src/nodes/launchNodes.ts:12-13", "N": 3, "F": 0, "init": [1, 1, 1], "faulty": [T, F_, F_],
     "error": "faultyList doesnt have F faulties"},
    {"src": "src/nodes/launchNodes.ts:12-13", "N": 3, "F": 2, "init": [1, 1, 1], "faulty": [T, F_, F_],
     "error": "faultyList doesnt have F faulties"},
]

SEED = 0x243F6A8885A308D3


def first_f(N, F):
    return [i < F for i in range(N)]


def state_cases():
    """Per-node final states: fixed-init cases (all inputs of small networks,
    plus tie-heavy ones) and random-init trials."""
    out = []
    # every 0/1 input of the reference's shapes
    shapes = [(5, 0, [F_] * 5), (5, 1, [F_, F_, F_, F_, T]), (7, 2, [F_, F_, T, F_, T, F_, F_]),
              (6, 2, [T, F_, F_, F_, F_, T]), (4, 0, [F_] * 4), (10, 4, first_f(10, 4))]
    for N, F, fl in shapes:
        live = [i for i in range(N) if not fl[i]]
        for bits in itertools.product([0, 1], repeat=len(live)):
            if N == 10 and sum(bits) not in (2, 3, 4):   # keep the file small, tie-rich
                continue
            init = [1] * N
            for i, b in zip(live, bits):
                init[i] = b
            out.append({"N": N, "F": F, "faulty": fl, "init": init, "seed": SEED, "trial": len(out), "k_max": 16})
    # '?' initial values (types.ts:8 allows them)
    out.append({"N": 5, "F": 1, "faulty": [F_, F_, F_, F_, T], "init": ["?", "?", 1, 0, 1], "seed": SEED,
                "trial": 9001, "k_max": 16})
    out.append({"N": 4, "F": 0, "faulty": [F_] * 4, "init": ["?", "?", "?", "?"], "seed": SEED, "trial": 9002,
                "k_max": 16})
    # no-decision shape (N <= 2F) with a tie-prone start
    out.append({"N": 10, "F": 5, "faulty": first_f(10, 5), "init": [0] * 5 + [0, 1, 0, 1, 1], "seed": SEED,
                "trial": 9003, "k_max": 11})
    out.append({"N": 8, "F": 4, "faulty": first_f(8, 4), "init": [0] * 4 + [0, 1, 0, 1], "seed": SEED,
                "trial": 9004, "k_max": 11})
    # random init trials on larger shapes (exercise W > 1 and block padding)
    for (N, F, ntr) in [(64, 0, 6), (130, 2, 6), (100, 30, 6), (1024, 341, 3), (1100, 40, 2), (200, 72, 6)]:
        for t in range(ntr):
            out.append({"N": N, "F": F, "faulty": first_f(N, F), "init": None, "seed": SEED + N,
                        "trial": 1000 + t, "k_max": 32})
    return out


HIST_CASES = [
    # (N, F, trials, k_max)
    (5, 1, 20000, 16), (10, 4, 20000, 16), (10, 5, 5000, 11), (7, 2, 5000, 16), (64, 0, 5000, 32),
    (100, 30, 3000, 32), (256, 85, 2000, 16), (1024, 341, 500, 16), (1100, 40, 200, 32),
    (4096, 0, 100, 16), (4096, 2048, 50, 16), (1, 0, 100, 4), (2, 0, 2000, 32),
]


RANDOM_HIST_CASES = [
    # (N, F, f, trials, k_max): random-delivery model, the first f nodes crashed
    (10, 4, 2, 20000, 16), (10, 4, 0, 20000, 16), (7, 3, 1, 20000, 16), (100, 30, 10, 2000, 16),
    (200, 90, 0, 500, 16), (70, 40, 0, 2000, 16), (130, 20, 5, 500, 16), (1100, 40, 20, 20, 16),
    (1024, 341, 0, 40, 16), (64, 10, 3, 1000, 16),
]

RANDOM_STATE_CASES = [(12, 4, 1), (10, 4, 2), (100, 30, 5), (70, 40, 0), (130, 40, 10)]


EVENT_HIST_CASES = [
    # (N, F, trials, k_max, crash_count, crash_window): event-level mode, first F nodes faulty
    (10, 4, 3000, 16, 0, 0), (10, 4, 3000, 16, 1, 150), (5, 1, 3000, 16, 1, 40), (16, 5, 1000, 16, 2, 400),
    (33, 10, 300, 16, 1, 2000), (64, 21, 100, 16, 3, 8000), (12, 4, 2000, 16, 0, 0), (7, 3, 2000, 12, 1, 60),
    # N > 64 (r02): node-id bitsets of 4 words
    (100, 30, 60, 16, 2, 20000), (128, 42, 40, 16, 3, 40000), (256, 85, 8, 16, 4, 150000), (130, 0, 40, 16, 0, 0),
]

EVENT_STATE_CASES = [
    # (N, F, init, crash_at (None = never), trial)
    (10, 4, [1] * 10, {7: 0}, 1), (10, 4, [1] * 10, {7: 60}, 7), (10, 4, [1] * 10, {7: 70}, 7),
    (5, 1, [1, 1, 1, 0, 0], {0: 5}, 2), (6, 2, [0, 1, 0, 1, 1, 0], {2: 12, 3: 30}, 3),
    (9, 4, [0, 0, 1, 1, 1, 0, 0, 1, 1], None, 4), (12, 4, [0, 1] * 6, {5: 100}, 5),
]


def encode_state(s):
    """NodeState -> [killed, x, decided, k] with null = -1 and '?' = 2."""
    x = {None: -1, 0: 0, 1: 1, "?": 2}[s["x"]]
    d = -1 if s["decided"] is None else int(s["decided"])
    k = -1 if s["k"] is None else s["k"]
    return [int(s["killed"]), x, d, k]


def decode_state(e):
    return {"killed": bool(e[0]), "x": {-1: None, 0: 0, 1: 1, 2: "?"}[e[1]],
            "decided": None if e[2] < 0 else bool(e[2]), "k": None if e[3] < 0 else e[3]}


def main():
    with open(os.path.join(HERE, "reference_cases.json"), "w") as f:
        json.dump({"source": "viviendbk/ben-or-consensus-algorithm " + TEST + ", src/nodes/launchNodes.ts",
                   "cases": REFERENCE_CASES, "launch_errors": LAUNCH_ERRORS}, f, indent=1)

    states = []
    for c in state_cases():
        init = c["init"]
        N, F = c["N"], c["F"]
        res = oracle.run_trials(N, F, c["faulty"], seed=c["seed"], trial_begin=c["trial"], trial_count=1,
                                k_max=c["k_max"], initial_values=init, want_states=True)
        if init is not None:
            r_msg, stalled, st_msg = oracle.message_sim(N, F, init, c["faulty"], seed=c["seed"],
                                                        trial=c["trial"], k_max=c["k_max"])
            assert not stalled
            assert st_msg == res.states, (c, st_msg, res.states)
        states.append({**c, "states": [encode_state(s) for s in res.states],
                       "hist_nonzero": {str(i): int(v) for i, v in enumerate(res.hist) if v}})

    hists = []
    for (N, F, ntr, k_max) in HIST_CASES:
        res = oracle.run_trials(N, F, first_f(N, F), seed=SEED ^ N, trial_begin=12345, trial_count=ntr, k_max=k_max)
        nz = {str(i): int(v) for i, v in enumerate(res.hist) if v}
        hists.append({"N": N, "F": F, "seed": SEED ^ N, "trial_begin": 12345, "trial_count": ntr, "k_max": k_max,
                      "hist_nonzero": nz})
    rhists = []
    for (N, F, f, ntr, k_max) in RANDOM_HIST_CASES:
        fl = first_f(N, f)
        res = oracle.run_trials(N, F, fl, seed=SEED ^ (N * 31 + f), trial_begin=777, trial_count=ntr, k_max=k_max,
                                mode=oracle.MODE_RANDOM_DELIVERY)
        rhists.append({"N": N, "F": F, "faulty": fl, "seed": SEED ^ (N * 31 + f), "trial_begin": 777,
                       "trial_count": ntr, "k_max": k_max,
                       "hist_nonzero": {str(i): int(v) for i, v in enumerate(res.hist) if v}})
    rstates = []
    for (N, F, f) in RANDOM_STATE_CASES:
        for t in range(4):
            fl = first_f(N, f)
            init = None if t % 2 else [int(b) for b in format((t * 2654435761) % (1 << N), f"0{N}b")[:N]]
            res = oracle.run_trials(N, F, fl, seed=SEED + t, trial_begin=50 + t, trial_count=1, k_max=24,
                                    initial_values=init, want_states=True, mode=oracle.MODE_RANDOM_DELIVERY)
            rstates.append({"N": N, "F": F, "faulty": fl, "init": init, "seed": SEED + t, "trial": 50 + t,
                            "k_max": 24, "states": [encode_state(x) for x in res.states]})
    ehists = []
    for (N, F, ntr, k_max, cc, cw) in EVENT_HIST_CASES:
        fl = first_f(N, F)
        res, ev = oracle.event_trials(N, F, fl, seed=SEED ^ (N * 131 + cc), trial_begin=99, trial_count=ntr,
                                      k_max=k_max, crash_count=cc, crash_window=cw)
        ehists.append({"N": N, "F": F, "faulty": fl, "seed": SEED ^ (N * 131 + cc), "trial_begin": 99,
                       "trial_count": ntr, "k_max": k_max, "crash_count": cc, "crash_window": cw, "events": ev,
                       "hist_nonzero": {str(i): int(v) for i, v in enumerate(res.hist) if v}})
    estates = []
    for (N, F, init, crashes, trial) in EVENT_STATE_CASES:
        fl = first_f(N, F)
        ca = None if crashes is None else [crashes.get(i) for i in range(N)]
        res, ev = oracle.event_trials(N, F, fl, seed=SEED, trial_begin=trial, trial_count=1, k_max=24,
                                      initial_values=init, crash_at=ca, want_states=True)
        estates.append({"N": N, "F": F, "faulty": fl, "init": init, "crash_at": ca, "seed": SEED, "trial": trial,
                        "k_max": 24, "events": ev, "states": [encode_state(x) for x in res.states],
                        "hist_nonzero": {str(i): int(v) for i, v in enumerate(res.hist) if v}})
    with open(os.path.join(HERE, "oracle_vectors.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (oracle/benor_oracle.c restatements (i)+(ii)+(iii))",
                   "states": states, "hists": hists, "random_hists": rhists, "random_states": rstates,
                   "event_hists": ehists, "event_states": estates}, f, separators=(",", ":"))
    print(f"{len(states)} state cases, {len(hists)} histograms, {len(rhists)} random-delivery histograms, "
          f"{len(rstates)} random-delivery state cases")


if __name__ == "__main__":
    main()
