"""Parity of the HIP path (via the C ABI) against the CPU oracle.  GPU only.

Bit-exact integer agreement is required everywhere:
* per-node final NodeState of every committed golden state case
  (tests/golden/oracle_vectors.json: every 0/1 input of the reference's
  shapes, '?' inputs, coin-heavy ties, W > 1 and padded tally blocks);
* outcome histograms of the committed golden histogram cases;
* fresh seeded batches against the oracle run live on the same inputs;
* the reference's own known-answer tests through the network API.
At BASELINE's full sizes (N=1024, F=341, up to 10^7 trials per launch),
size-independent properties: sharding invariance (histogram of [0, T) equals
the sum over any split), R == 1 whenever m is odd, agreement, and the exact
analytic law by chi-square.
"""
import itertools

import os

import numpy as np
import pytest

import analytic
import benor
import oracle
from conftest import check_reference_expectations
from make_golden import decode_state

pytestmark = pytest.mark.gpu


def first_f(N, F):
    return [i < F for i in range(N)]


def test_golden_states(oracle_vectors):
    for c in oracle_vectors["states"]:
        rounds, st = benor.run_trial_states(c["N"], c["F"], c["faulty"], seed=c["seed"], trial=c["trial"],
                                            k_max=c["k_max"], initial_values=c["init"])
        assert st == [decode_state(e) for e in c["states"]], c


def test_golden_histograms(oracle_vectors):
    for h in oracle_vectors["hists"]:
        plan = benor.TrialsPlan(h["N"], h["F"], first_f(h["N"], h["F"]), seed=h["seed"], k_max=h["k_max"])
        got = plan.run(h["trial_begin"], h["trial_count"])
        assert {str(i): int(v) for i, v in enumerate(got) if v} == h["hist_nonzero"], (h["N"], h["F"])


@pytest.mark.parametrize("N,F,trials,k_max", [
    (10, 4, 200_000, 24), (10, 5, 50_000, 11), (5, 1, 100_000, 24), (64, 0, 30_000, 32),
    (70, 2, 20_000, 32), (128, 0, 20_000, 32), (256, 85, 20_000, 16), (1024, 341, 5_000, 16),
    (1088, 0, 500, 32), (1100, 40, 1_000, 32), (2047, 0, 200, 32), (4096, 0, 100, 16), (4096, 2047, 100, 16),
    (3, 1, 10_000, 8), (1, 0, 1000, 4), (2, 1, 1000, 4), (33, 16, 5000, 16),
    # even m at W = 5, 8, 16: multi-round trials through the fused next-round R-phase
    (300, 0, 4000, 24), (600, 100, 3000, 24), (1024, 0, 2000, 24),
    # m <= F, W = 1, 2, 8: never decide, every trial runs to k_max
    (100, 50, 2000, 12), (200, 100, 1000, 12), (1000, 500, 100, 12),
    # k_max = BO_MAX_K: histogram of 3076 bins (bins >= 64 through LDS atomics)
    (10, 5, 500, 1024), (130, 65, 100, 1024), (2, 0, 20000, 1024), (70, 4, 3000, 1024),
])
def test_random_batches_match_oracle(N, F, trials, k_max):
    seed = 0x9E3779B97F4A7C15 ^ (N * 7919 + F)
    plan = benor.TrialsPlan(N, F, first_f(N, F), seed=seed, k_max=k_max)
    got = plan.run(777, trials)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=777, trial_count=trials, k_max=k_max)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.parametrize("N,F,reps", [(12, 4, 30), (16, 6, 30), (9, 3, 30), (64, 2, 30),
                                      # per-node state from the W kernel at W = 17, 32 and the blocked kernel
                                      (1090, 2, 4), (2047, 1, 3), (2600, 300, 3), (4096, 0, 2)])
def test_random_fault_placement_states(N, F, reps):
    """Fault placement is arbitrary (faultyList); per-node states must match."""
    rng = np.random.default_rng(N + 31 * F)
    for t in range(reps):
        fl = [False] * N
        for i in rng.choice(N, F, replace=False):
            fl[i] = True
        init = [int(v) for v in rng.integers(0, 2, N)]
        if N > 1000 and t % 2 == 1:        # tied start (m even): round 1 proposes "?", coins decide
            live = [i for i in range(N) if not fl[i]]
            ones = set(int(i) for i in rng.choice(live, len(live) // 2, replace=False))
            init = [1 if i in ones else 0 for i in range(N)]
        seed = int(rng.integers(0, 2**63))
        ref = oracle.run_trials(N, F, fl, seed=seed, trial_begin=t, trial_count=1, k_max=20,
                                initial_values=init, want_states=True).states
        _, got = benor.run_trial_states(N, F, fl, seed=seed, trial=t, k_max=20, initial_values=init)
        assert got == ref


@pytest.mark.parametrize("N,F,W,G", [(2113, 0, 34, 17), (2800, 0, 44, 22), (4000, 0, 63, 21), (2600, 300, 36, 18)])
def test_blocked_kernel_block_sizes(N, F, W, G):
    """The blocked kernel (m > 2048) at block sizes G > 16, where even-M
    proposal records are staged in two VGPRs: random-init histograms and a
    tied fixed start (round 1 proposes "?", coins follow) per node, against
    the oracle.  W = ceil(m/64); G is the plan's block size."""
    m = N - F
    assert (m + 63) // 64 == W
    seed = 0xB10C ^ N
    plan = benor.TrialsPlan(N, F, first_f(N, F), seed=seed, k_max=24)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=11, trial_count=300, k_max=24)
    np.testing.assert_array_equal(plan.run(11, 300), ref.hist)
    if m % 2 == 0:
        live = [i for i in range(N) if i >= F]
        init = [0] * N
        for i in live[::2]:
            init[i] = 1                                  # m/2 ones: tied round 1
        for t in range(2):
            want = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=t, trial_count=1, k_max=24,
                                     initial_values=init, want_states=True).states
            _, got = benor.run_trial_states(N, F, first_f(N, F), seed=seed, trial=t, k_max=24, initial_values=init)
            assert got == want


def test_reference_known_answers_network_api(reference_cases):
    """benorconsensus.test.ts:133-486 through launchNetwork / startConsensus /
    getNodesState / stopConsensus -- the reference's call sequence."""
    for case in reference_cases["cases"]:
        inits = ([list(b) for b in itertools.product([0, 1], repeat=case["N"])]
                 if case["init"] == "random01" else [case["init"]])
        for init in inits:
            N = case["N"]
            servers = benor.launchNetwork(N, sum(case["faulty"]), init, case["faulty"])
            statuses = [benor.getStatus(i) for i in range(N)]
            if case["start"]:
                benor.startConsensus(N, seed=0x5EED)
                benor.waitConsensus(N)
                states = benor.getNodesState(N)
                assert benor.reachedFinality(states) or any(s["decided"] is False for s in states)
                check_reference_expectations(case, states)
                ref = oracle.run_trials(N, sum(case["faulty"]), case["faulty"], seed=0x5EED, trial_begin=0,
                                        trial_count=1, k_max=benor.DEFAULT_K_MAX, initial_values=init,
                                        want_states=True).states
                if all(r["decided"] is True for r in ref):          # auto-stop (node.ts:116-145)
                    ref = [dict(r, killed=True) for r in ref]
                assert states == ref
            else:
                check_reference_expectations(case, benor.getNodesState(N), statuses)
            benor.stopConsensus(N)
            assert all(benor.getStatus(i)[0] == 500 for i in range(N))
            for s in servers:
                s.close()


def test_stopped_nodes_stall():
    """A node stopped before start leaves fewer than N-F senders: the round-1
    R-phase never triggers (node.ts:52), so live nodes sit at k = 1."""
    servers = benor.launchNetwork(5, 1, [1, 1, 1, 0, 0], [False, False, False, False, True])
    servers[0]._net.stop_node(0)
    benor.startConsensus(5, seed=3)
    st = benor.getNodesState(5)
    assert st[0]["killed"] and st[0]["k"] == 0
    assert all(s["k"] == 1 and s["decided"] is False for s in st[1:4])


def test_second_start_is_a_no_op():
    """The reference's round inboxes (node.ts:29-30) outlive a run, so a second
    GET /start re-triggers every round-1 tally (node.ts:47-52) instead of
    running a fresh consensus.  startConsensus resolves as the reference's does
    (every /start answers 200) and runs nothing: the first run's states stay;
    the C ABI (and strict=True) reports BO_ERR_ALREADY_STARTED."""
    benor.launchNetwork(6, 2, [0, 0, 1, 1, 0, 1], [True, False, False, False, False, True])
    benor.startConsensus(6, seed=1)
    benor.waitConsensus(6)
    a = benor.getNodesState(6)
    benor.startConsensus(6, seed=2)
    assert benor.getNodesState(6) == a and all(s["decided"] for s in a[1:5])
    with pytest.raises(benor.AlreadyStartedError, match="already started"):
        benor.startConsensus(6, seed=1, strict=True)


def test_stop_during_run_is_kept():
    """A /stop served while a sync start's kernel runs (another thread) is
    ordered after the run: the node keeps its final state and stays killed.  N=2048 with
    F=1024 never decides (m <= 2F), so the run lasts k_max = 1024 rounds."""
    import threading

    N, F, K = 2048, 1024, 1024
    init = [i % 2 for i in range(N)]
    benor.launchNetwork(N, F, init, [i < F for i in range(N)])
    net = benor._current
    t = threading.Thread(target=lambda: benor.startConsensus(N, seed=9, k_max=K, sync=True))
    t.start()
    net.stop_node(1500)
    t.join()
    st = benor.getNodesState(N)
    assert st[1500]["killed"] is True and all(not s["killed"] for i, s in enumerate(st) if i >= F and i != 1500)
    if st[1500]["k"] == 0:     # served before the start: 1023 < N - F senders, a stall (node.ts:52)
        assert all(s["k"] == 1 and s["decided"] is False for i, s in enumerate(st) if i >= F and i != 1500)
    else:                      # served during (or after) the run: node 1500 keeps its final state
        assert st[1500]["k"] == st[F]["k"] == K + 1 and st[1500]["decided"] is False


def test_auto_stop_kills_every_node_when_all_decided():
    """node.ts:116-145: once every node's /getState reports decided, every node
    gets /stop.  Faulty nodes report decided: null, so it fires only at F = 0
    (and without nodes stopped before the run)."""
    benor.launchNetwork(5, 0, [1, 1, 0, 1, 1], [False] * 5)
    benor.startConsensus(5, seed=4)
    benor.waitConsensus(5)
    st = benor.getNodesState(5)
    assert all(s["killed"] and s["decided"] and s["x"] == 1 and s["k"] == 2 for s in st)
    assert all(benor.getStatus(i) == (500, "faulty") for i in range(5))
    benor.launchNetwork(5, 1, [1, 1, 0, 1, 1], [False] * 4 + [True])
    benor.startConsensus(5, seed=4)
    benor.waitConsensus(5)
    assert not any(s["killed"] for s in benor.getNodesState(5)[:4])


@pytest.mark.parametrize("N,F", [
    # odd m (odd-only kernel, K = 16 / 8 / 8 / 8 / 3 / 2): every receiver decides ...
    (64, 21), (128, 41), (256, 85), (300, 71), (400, 100), (600, 151),
    # ... or not (m <= 2F: undecided trials re-run alone after the interleaved round 1)
    (100, 49), (200, 99),
    # even m (K = 8 / 8 / 4 / 4 / 3): ties, coins and re-runs
    (64, 20), (128, 42), (256, 86), (300, 72), (512, 170),
])
def test_interleaved_round1_matches_oracle(N, F):
    """The W kernel runs round 1 of K trials interleaved only when a wave holds
    K trials of the launch, i.e. at trial counts of about K x the grid's wave
    count (8 per CU x 4 waves x 256 CUs): 200 000 trials engage every K here
    (`interleave_k`).  Bit-identical to the oracle."""
    seed = 0xB5AD4ECEDA1CE2A9 ^ (N * 131 + F)
    plan = benor.TrialsPlan(N, F, first_f(N, F), seed=seed, k_max=16)
    T = 200_000
    got = plan.run(31, T)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=31, trial_count=T, k_max=16)
    np.testing.assert_array_equal(got, ref.hist)
    np.testing.assert_array_equal(got, plan.run(31, 70_001) + plan.run(70_032, T - 70_001))


# ------------------------------------------------- full-size properties
def test_full_size_sharding_invariance_and_law():
    """N=1024, F=341 (BASELINE metric config): m = 683 is odd, so no round can
    tie -- every trial decides the live majority in round 1.  The
    histogram of one launch equals the sum of a split run (global Philox
    counters), and the decided value is Bernoulli(1/2)."""
    N, F, k = 1024, 341, 16
    plan = benor.TrialsPlan(N, F, first_f(N, F), seed=0x243F6A8885A308D3, k_max=k)
    T = 2_000_000
    whole = plan.run(0, T)
    parts = plan.run(0, 600_001) + plan.run(600_001, 1_000_000) + plan.run(1_600_001, T - 1_600_001)
    np.testing.assert_array_equal(whole, parts)
    assert whole.sum() == T
    assert whole[3] + whole[4] == T            # bins (R=1, v=0), (R=1, v=1)
    assert whole[-1] == 0
    assert analytic.chi2_pvalue(whole[:-1], analytic.hist_probs(N, F, k)) > 0.01
    # a spot-check of the same launch range against the oracle
    ref = oracle.run_trials(N, F, first_f(N, F), seed=0x243F6A8885A308D3, trial_begin=1_999_000,
                            trial_count=1000, k_max=k)
    np.testing.assert_array_equal(plan.run(1_999_000, 1000), ref.hist)


@pytest.mark.parametrize("N,F,T", [(10, 4, 1_000_000), (5, 1, 300_000), (64, 21, 500_000), (10, 5, 200_000),
                                   (256, 0, 2_000_000), (2048, 0, 100_000)])
def test_histogram_independent_of_grid(N, F, T):
    """The grid a launch gets (workgroups per CU: the lane kernel's short-launch
    rule, LDS fit, the matrix-core continuation passes) only decides which wave
    runs which trial ids: BENOR_BLOCKS_PER_CU = 1 or 3 gives the histogram of
    the default grid, bit for bit."""
    fl = first_f(N, F)
    base = benor.TrialsPlan(N, F, fl, seed=4242, k_max=16).run(11, T)
    for bpc in ("1", "3"):
        os.environ["BENOR_BLOCKS_PER_CU"] = bpc
        try:
            got = benor.TrialsPlan(N, F, fl, seed=4242, k_max=16).run(11, T)
        finally:
            os.environ.pop("BENOR_BLOCKS_PER_CU", None)
        np.testing.assert_array_equal(got, base)
    assert base[:-1].sum() == T


def test_launch_split_past_2_31_trials():
    """The host splits launches at 2^31 trials (the kernels index trials within
    a launch in 32 bits): a 2^31 + 3000-trial run loses no trial, its last
    3000 trials equal a separate launch of that range, and m = 39 (odd) halts
    every trial in round 1 with a Bernoulli(1/2) value."""
    N, F, k = 40, 1, 8
    plan = benor.TrialsPlan(N, F, first_f(N, F), seed=77, k_max=k)
    T = (1 << 31) + 3000
    h = plan.run(5, T)
    assert h.sum() == T and h[3] + h[4] == T
    assert analytic.chi2_pvalue(h[:-1], analytic.hist_probs(N, F, k)) > 0.01
    tail = plan.run(5 + (1 << 31), 3000)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=77, trial_begin=5 + (1 << 31), trial_count=3000, k_max=k)
    np.testing.assert_array_equal(tail, ref.hist)


# north_star: in random mode the rounds-to-decide and decided-value
# distributions pass KS / chi-square at p > 0.01 against the reference network's
# law, including the F > N/2 no-decision case
# (benorconsensus.test.ts:292-345).  10^6 trials each (BASELINE configs[1]).
P_MIN = 0.01


@pytest.mark.parametrize("N,F,k_max", [(5, 1, 24), (10, 4, 24), (10, 5, 11), (64, 0, 32), (100, 30, 32),
                                       (12, 6, 16), (256, 86, 16)])
def test_analytic_law_1e6(N, F, k_max):
    plan = benor.TrialsPlan(N, F, first_f(N, F), seed=0xA11CE + N, k_max=k_max)
    h = plan.run(0, 1_000_000)
    assert h.sum() == 1_000_000 and h[-1] == 0
    probs = analytic.hist_probs(N, F, k_max)
    assert analytic.chi2_pvalue(h[:-1], probs) > P_MIN            # joint (rounds, decided value)
    assert analytic.ks_rounds_pvalue(h[:-1], probs, k_max) > P_MIN  # rounds-to-decision CDF
    decided = h[3:-1].reshape(-1, 3).sum(axis=0)                   # decided-value marginal
    if decided[:2].sum():
        pv = analytic.chi2_pvalue(decided[:2], np.array([0.5, 0.5]))
        assert pv > P_MIN and decided[2] == 0


def test_no_decision_case_f_gt_half():
    """Exceeding Fault Tolerance (benorconsensus.test.ts:292-345) at scale:
    N=10, F=5 never decides; every trial runs k_max rounds (k = k_max+1 > 10)."""
    plan = benor.TrialsPlan(10, 5, first_f(10, 5), seed=5, k_max=11)
    h = plan.run(0, 1_000_000)
    assert h[:3].sum() == 1_000_000


def test_popc_peak_probe_runs():
    peak = benor.popc_peak(5)
    assert peak > 1e12


# ------------------------------------------------- random delivery (f <= F)
RD = benor.BO_MODE_RANDOM_DELIVERY


def test_random_delivery_golden(oracle_vectors):
    for h in oracle_vectors["random_hists"]:
        plan = benor.TrialsPlan(h["N"], h["F"], h["faulty"], seed=h["seed"], k_max=h["k_max"], mode=RD)
        got = plan.run(h["trial_begin"], h["trial_count"])
        assert {str(i): int(v) for i, v in enumerate(got) if v} == h["hist_nonzero"], (h["N"], h["F"])
    for c in oracle_vectors["random_states"]:
        _, st = benor.run_trial_states(c["N"], c["F"], c["faulty"], seed=c["seed"], trial=c["trial"],
                                       k_max=c["k_max"], initial_values=c["init"], mode=RD)
        assert st == [decode_state(e) for e in c["states"]], c


@pytest.mark.parametrize("N,F,f,trials", [(10, 4, 1, 100_000), (9, 4, 0, 100_000), (66, 20, 3, 3000),
                                          (300, 120, 40, 200), (2100, 700, 0, 3), (4096, 1365, 1000, 2)])
def test_random_delivery_matches_oracle(N, F, f, trials):
    fl = first_f(N, f)
    seed = 0x51ED ^ N ^ (f << 16)
    got = benor.TrialsPlan(N, F, fl, seed=seed, k_max=16, mode=RD).run(5, trials)
    ref = oracle.run_trials(N, F, fl, seed=seed, trial_begin=5, trial_count=trials, k_max=16,
                            mode=oracle.MODE_RANDOM_DELIVERY)
    np.testing.assert_array_equal(got, ref.hist)


# Bernoulli + fix-up sampler (k >= 64, 8k > m): every comparator width (a odd,
# a = 2 mod 4, a = 4 mod 8, a = 8: 4, 3, 2, 1 stream words per mask word), every
# index-field width class (b = 7..12: 4, 3 or 2 fields per word; b = 7 only at
# m = 128, q = 64) and m = 2^b (no range check) against the oracle.
@pytest.mark.parametrize("m,q", [(256, 170), (200, 120), (512, 380), (700, 315), (1024, 683), (1500, 1003),
                                 (3000, 1790), (2048, 1229), (256, 66), (128, 64)])
def test_random_delivery_bernoulli_sampler_shapes(m, q):
    ab = oracle.delivery_bernoulli(m, q)
    assert ab is not None
    f = 3 if m < 1024 else 0                       # crashed nodes: N = m + f, quorum q = N - F
    N, F = m + f, m + f - q
    fl = first_f(N, f)
    seed = 0xBE5 ^ m ^ (q << 13)
    T = 40 if m >= 1500 else 200
    got = benor.TrialsPlan(N, F, fl, seed=seed, k_max=8, mode=RD).run(17, T)
    ref = oracle.run_trials(N, F, fl, seed=seed, trial_begin=17, trial_count=T, k_max=8,
                            mode=oracle.MODE_RANDOM_DELIVERY)
    np.testing.assert_array_equal(got, ref.hist)


def test_random_delivery_equals_lockstep_at_f_equals_F():
    for N, F in [(10, 4), (100, 33), (1024, 341)]:
        fl = first_f(N, F)
        a = benor.TrialsPlan(N, F, fl, seed=3, k_max=16, mode=RD).run(0, 20_000)
        b = benor.TrialsPlan(N, F, fl, seed=3, k_max=16).run(0, 20_000)
        np.testing.assert_array_equal(a, b)


def test_random_delivery_rejects_too_many_faults():
    with pytest.raises(benor.Error):
        benor.TrialsPlan(10, 2, first_f(10, 3), mode=RD)


# ------------------------------------------------- event-level mode (N <= 256)
EV = benor.BO_MODE_EVENT


def test_event_mode_golden(oracle_vectors):
    for h in oracle_vectors["event_hists"]:
        plan = benor.TrialsPlan(h["N"], h["F"], h["faulty"], seed=h["seed"], k_max=h["k_max"], mode=EV,
                                crash_count=h["crash_count"], crash_window=h["crash_window"])
        got = plan.run(h["trial_begin"], h["trial_count"])
        assert {str(i): int(v) for i, v in enumerate(got) if v} == h["hist_nonzero"], (h["N"], h["crash_count"])
    for c in oracle_vectors["event_states"]:
        _, st = benor.run_trial_states(c["N"], c["F"], c["faulty"], seed=c["seed"], trial=c["trial"],
                                       k_max=c["k_max"], initial_values=c["init"], mode=EV, crash_at=c["crash_at"])
        assert st == [decode_state(e) for e in c["states"]], c


@pytest.mark.parametrize("N,F,cc,cw,trials", [(10, 4, 0, 0, 200_000), (10, 4, 1, 150, 200_000),
                                              (20, 6, 2, 600, 20_000), (64, 21, 4, 10_000, 500),
                                              (3, 1, 1, 6, 50_000), (1, 0, 0, 0, 1000),
                                              # inbox counters in LDS up to N = 31 (5-bit fields), then scratch
                                              (16, 5, 1, 300, 20_000), (31, 10, 3, 2_000, 5_000),
                                              (32, 10, 2, 2_000, 3_000), (29, 0, 2, 1_500, 5_000),
                                              # N > 64 (r02): 4-word node bitsets, 8-bit node ids
                                              (65, 20, 2, 9_000, 300), (128, 42, 3, 40_000, 200),
                                              (256, 85, 5, 150_000, 20), (200, 0, 1, 80_000, 20)])
def test_event_mode_matches_oracle(N, F, cc, cw, trials):
    fl = first_f(N, F)
    seed = 0xE7E7 ^ N
    got = benor.TrialsPlan(N, F, fl, seed=seed, k_max=16, mode=EV, crash_count=cc, crash_window=cw).run(3, trials)
    ref, _ = oracle.event_trials(N, F, fl, seed=seed, trial_begin=3, trial_count=trials, k_max=16,
                                 crash_count=cc, crash_window=cw)
    np.testing.assert_array_equal(got, ref.hist)


def test_event_mode_without_stop_equals_lockstep_kernel():
    for N, F in [(10, 4), (64, 21), (33, 0), (128, 42), (100, 0), (31, 10), (17, 0)]:
        fl = first_f(N, F)
        a = benor.TrialsPlan(N, F, fl, seed=8, k_max=16, mode=EV).run(0, 50_000)
        b = benor.TrialsPlan(N, F, fl, seed=8, k_max=16).run(0, 50_000)
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("N,F,f,T,init", [(1024, 341, 0, 400, None), (1024, 341, 100, 300, None),
                                          (600, 200, 37, 600, "q"), (4096, 1365, 0, 24, None),
                                          (3000, 1210, 0, 40, None), (257, 80, 1, 2000, "q")])
def test_random_delivery_bernoulli_kernel_matches_oracle(N, F, f, T, init):
    """The Bernoulli-sampler kernel (benor_random.hip: uniform Philox rounds
    hoisted, ds_mskor_rtn fix-up with speculative batches and undo, padded
    bitset rows) against oracle_delivery_mask's sequential definition, on
    random and fixed initial values with "?" inputs.  (Until r04 this compared
    it with the r02 kernel, which r05 deleted.)"""
    fl = first_f(N, f)
    vals = None
    if init == "q":
        rng = np.random.default_rng(N)
        vals = ["?" if rng.random() < 0.1 else int(rng.integers(0, 2)) for _ in range(N)]
    plan = benor.TrialsPlan(N, F, fl, seed=0xA5A5 ^ N, k_max=12, mode=RD, initial_values=vals)
    assert plan.kernel == benor.BO_KERNEL_RANDOM
    ref = oracle.run_trials(N, F, fl, seed=0xA5A5 ^ N, trial_begin=99, trial_count=T, k_max=12,
                            mode=oracle.MODE_RANDOM_DELIVERY, initial_values=vals)
    np.testing.assert_array_equal(plan.run(99, T), ref.hist)


# ------------------------------------- event level above N = 256 (benor_event_big.hip)
@pytest.mark.parametrize("N,F,trials,stops,init", [
    (257, 0, 6, None, None), (300, 100, 5, {150: 20_000, 299: 55_000}, None), (512, 170, 3, None, "tied"),
    (700, 233, 2, {300: 100}, None), (1000, 0, 2, None, None), (513, 256, 2, None, None)])
def test_event_mode_big_matches_oracle(N, F, trials, stops, init):
    """One wave per trial (256 < N <= 4096): histograms of several trials
    (batched speculative picks, overlay write-back, triggers mid-batch, stops at
    batch boundaries) equal oracle (iii) event_trial; with fixed tied starts the
    runs reach round 2 through coins; F = N/2 - ... (513, 256) cannot decide."""
    fl = first_f(N, F)
    seed = 0xB16 ^ N
    sched = None
    if stops:
        sched = [None] * N
        for node, e in stops.items():
            sched[node] = e
    vals = None
    if init == "tied":
        m = N - F
        vals = [0] * F + [i % 2 for i in range(m)]
    got = benor.TrialsPlan(N, F, fl, seed=seed, k_max=8, mode=EV, crash_at=sched, initial_values=vals).run(7, trials)
    ref, _ = oracle.event_trials(N, F, fl, seed=seed, trial_begin=7, trial_count=trials, k_max=8, crash_at=sched,
                                 initial_values=vals)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.parametrize("N,F,cc,cw,trials", [(1024, 341, 1, 1_400_000, 3), (1024, 341, 3, 3_000_000, 3),
                                              (1024, 341, 5, 800_000, 2), (4096, 1365, 2, 23_000_000, 2),
                                              (4096, 1365, 5, 30_000_000, 1), (300, 99, 4, 180_000, 4)])
def test_event_mode_big_random_stops_match_oracle(N, F, cc, cw, trials):
    """A random /stop schedule (crash_count nodes at uniform delivery counts in
    [0, crash_window), drawn per trial from Philox stream 4) at the configs[3]
    and configs[4] shapes: the wave-per-trial kernel draws it on the device
    (Floyd picks, then one delivery count per pick) and its histograms equal
    oracle (iii) event_trials bit for bit.  Windows of about one to two rounds
    of deliveries put the stops inside rounds 1 and 2."""
    fl = first_f(N, F)
    seed = 0x5707 ^ N ^ (cc << 20)
    plan = benor.TrialsPlan(N, F, fl, seed=seed, k_max=8, mode=EV, crash_count=cc, crash_window=cw)
    assert plan.kernel == benor.BO_KERNEL_EVENT
    got = plan.run(11, trials)
    ref, _ = oracle.event_trials(N, F, fl, seed=seed, trial_begin=11, trial_count=trials, k_max=8,
                                 crash_count=cc, crash_window=cw)
    np.testing.assert_array_equal(got, ref.hist)


def test_event_mode_big_without_stop_equals_lockstep_kernel():
    """Without a /stop every phase completes with the whole live set, so the
    delivery order cannot change a tally: the big event kernel's histogram is
    the lockstep kernel's."""
    for N, F in [(300, 99), (1024, 341), (600, 0)]:
        fl = first_f(N, F)
        a = benor.TrialsPlan(N, F, fl, seed=9, k_max=16, mode=EV).run(0, 40)
        b = benor.TrialsPlan(N, F, fl, seed=9, k_max=16).run(0, 40)
        np.testing.assert_array_equal(a, b)


def test_event_mode_big_states_match_oracle():
    """Per-node states of one trial (bo_run_trial_states, the network API's
    launch) at N = 1024 with two scheduled stops in round 1."""
    N, F = 1024, 341
    fl = first_f(N, F)
    sched = [None] * N
    sched[400], sched[900] = 120_000, 700_000
    _, st = benor.run_trial_states(N, F, fl, seed=77, trial=0, k_max=16, mode=EV, crash_at=sched)
    ref, _ = oracle.event_trials(N, F, fl, seed=77, trial_begin=0, trial_count=1, k_max=16, crash_at=sched,
                                 want_states=True)
    assert st == ref.states
