"""Pin the CPU oracle before trusting it (CPU only).

* Philox4x32-10 against the Random123 known-answer vectors.
* The reference's launch validation (launchNodes.ts:10-13).
* Every known-answer test of the reference suite
  (__test__/tests/benorconsensus.test.ts:45-486) through both restatements.
* Message-level (i) == bit-plane (ii) on tie-heavy seeded cases, under FIFO
  and seeded-random delivery orders.
* The exact analytic outcome law by chi-square.
* The committed golden vectors are reproduced.
"""
import itertools

import numpy as np
import pytest

import analytic
import oracle
from conftest import check_reference_expectations
from make_golden import decode_state

# Random123 kat_vectors, philox4x32_10
PHILOX_KAT = [
    ([0, 0], [0, 0, 0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF, 0xFFFFFFFF], [0xFFFFFFFF] * 4, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0xA4093822, 0x299F31D0], [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


@pytest.mark.parametrize("key,ctr,out", PHILOX_KAT)
def test_philox_kat(key, ctr, out):
    assert oracle.philox4x32_10(key, ctr) == out


def test_coin_definition():
    """coin(c, r) = bit c & 31 of word (r-1) & 3 of Philox(ctr {trial, c >> 5,
    (r-1) >> 2}): the stand-in for Math.random() > 0.5 ? 0 : 1 (node.ts:111)."""
    for trial in range(20):
        for c in (0, 5, 31, 32, 70):
            for r in (1, 2, 4, 5, 9):
                b = oracle.philox4x32_10([0x1234, 0], [trial, 0, c >> 5, (r - 1) >> 2])
                assert oracle.coin(0x1234, trial, c, r) == (b[(r - 1) & 3] >> (c & 31)) & 1
    bits = [oracle.coin(7, t, c, r) for t in range(200) for c in range(40) for r in range(1, 9)]
    assert abs(sum(bits) / len(bits) - 0.5) < 0.01


def test_random_init_definition():
    """Random initial values: a network of m <= 32 live
    nodes takes bit c of word t & 3 of Philox(ctr {t >> 2, 1 << 31, 1 << 24}),
    so trials 4q .. 4q + 3 are the four words of one block; larger networks
    take bit c & 31 of word c >> 5 of the trial's own blocks
    (ctr {t, (c >> 5) >> 2, 1 << 24})."""
    key = [0x2468ACE1, 0x13579BDF]
    seed = key[0] | key[1] << 32
    for t in (0, 1, 2, 3, 4, 7, (1 << 33) + 5):
        q = t >> 2
        blk = oracle.philox4x32_10(key, [q & 0xFFFFFFFF, q >> 32, 1 << 31, 1 << 24])
        for m in (1, 6, 32):
            for c in range(m):
                assert oracle.random_init(seed, t, c, m) == (blk[t & 3] >> c) & 1
        for m in (33, 200):
            for c in (0, 31, 32, m - 1):
                b = oracle.philox4x32_10(key, [t & 0xFFFFFFFF, t >> 32, (c >> 5) >> 2, 1 << 24])
                assert oracle.random_init(seed, t, c, m) == (b[(c >> 5) & 3] >> (c & 31)) & 1
    bits = [oracle.random_init(11, t, c, 6) for t in range(4000) for c in range(6)]
    assert abs(sum(bits) / len(bits) - 0.5) < 0.01


def test_launch_errors(reference_cases):
    for e in reference_cases["launch_errors"]:
        code = oracle.validate(e["N"], e["F"], e["init"], e["faulty"])
        assert code == {"Arrays don't match": 1, "faultyList doesnt have F faulties": 2}[e["error"]]


def _run_case_message(case, init, seed=7):
    N = case["N"]
    F = sum(case["faulty"])
    return oracle.message_sim(N, F, init, case["faulty"], seed=seed, trial=0, k_max=64)


def _run_case_planes(case, init, seed=7):
    N = case["N"]
    F = sum(case["faulty"])
    return oracle.run_trials(N, F, case["faulty"], seed=seed, trial_begin=0, trial_count=1, k_max=64,
                             initial_values=init, want_states=True).states


def test_reference_known_answers(reference_cases):
    for case in reference_cases["cases"]:
        if not case["start"]:
            continue
        inits = ([list(b) for b in itertools.product([0, 1], repeat=case["N"])]
                 if case["init"] == "random01" else [case["init"]])
        for init in inits:
            r, stalled, st_i = _run_case_message(case, init)
            assert not stalled
            st_ii = _run_case_planes(case, init)
            assert st_i == st_ii
            check_reference_expectations(case, st_i)


@pytest.mark.parametrize("N,F", [(4, 0), (6, 2), (8, 2), (10, 4), (12, 4), (8, 4), (6, 3), (2, 0), (16, 6)])
def test_message_level_equals_bitplanes(N, F):
    """(i) == (ii) per node, including coin rounds: tie-heavy even-m shapes."""
    rng = np.random.default_rng(N * 100 + F)
    for t in range(40):
        faulty = [False] * N
        for i in rng.choice(N, F, replace=False):
            faulty[i] = True
        init = [int(v) for v in rng.integers(0, 2, N)]
        if t % 7 == 0:
            init[rng.integers(0, N)] = "?"
        seed = int(rng.integers(0, 2**63))
        for order in (0, 1):
            r, stalled, st_i = oracle.message_sim(N, F, init, faulty, seed=seed, trial=t, k_max=24,
                                                  order_mode=order)
            st_ii = oracle.run_trials(N, F, faulty, seed=seed, trial_begin=t, trial_count=1, k_max=24,
                                      initial_values=init, want_states=True).states
            assert st_i == st_ii, (N, F, init, faulty, order)


def test_delivery_order_independence():
    """With exactly F crashes every inbox is the full live set, so the seeded
    delivery order cannot change any outcome."""
    N, F = 9, 3
    faulty = [True] * F + [False] * (N - F)
    init = [0, 0, 0, 1, 1, 1, 0, 1, 0]
    ref = oracle.message_sim(N, F, init, faulty, seed=11, trial=5, order_mode=0)
    for salt in range(1, 30):
        got = oracle.message_sim(N, F, init, faulty, seed=11, trial=5, order_mode=salt)
        assert got == ref


def test_stall_when_fewer_live_than_quorum():
    # launchNodes accepts only exactly-F faults, but a node stopped before the
    # run leaves fewer senders than N-F: nothing ever triggers (node.ts:52).
    N, F = 5, 1
    r, stalled, st = oracle.message_sim(N, F, [1, 1, 1, 1, 1], [True, True, False, False, False], k_max=8)
    assert stalled and r == -1
    assert all(s["k"] == 1 and s["decided"] is False for s in st[2:])


@pytest.mark.parametrize("N,F,k_max", [(10, 4, 16), (5, 1, 16), (10, 5, 11), (64, 0, 24), (100, 30, 24),
                                       (7, 2, 16), (4, 1, 24), (12, 6, 12)])
def test_analytic_law(N, F, k_max):
    faulty = [i < F for i in range(N)]
    r = oracle.run_trials(N, F, faulty, seed=0xC0FFEE + N, trial_count=100000, k_max=k_max)
    probs = analytic.hist_probs(N, F, k_max)
    assert r.hist[-1] == 0                              # agreement never violated
    assert abs(probs.sum() - 1.0) < 1e-9
    # north_star: rounds-to-decide and decided-value distributions pass KS / chi-square at p > 0.01
    assert analytic.chi2_pvalue(r.hist[:-1], probs) > 0.01
    assert analytic.ks_rounds_pvalue(r.hist[:-1], probs, k_max) > 0.01


def test_ks_rejects_a_wrong_law():
    """The KS test has power: the N=10, F=4 histogram against the N=5, F=1 law
    (q = 0.3125 vs 0.375) is rejected."""
    r = oracle.run_trials(10, 4, [i < 4 for i in range(10)], seed=3, trial_count=100000, k_max=16)
    assert analytic.ks_rounds_pvalue(r.hist[:-1], analytic.hist_probs(5, 1, 16), 16) < 1e-6
    assert analytic.ks_rounds_pvalue(r.hist[:-1], analytic.hist_probs(10, 4, 16), 16) > 0.01


def test_expected_rounds_closed_form():
    # N=5,F=1 -> q=0.375, E[R]=1.6; N=10,F=4 -> q=0.3125, E[R]=1.4545
    assert analytic.tie_prob(4) == pytest.approx(0.375)
    assert analytic.expected_rounds(5, 1) == pytest.approx(1.6)
    assert analytic.tie_prob(6) == pytest.approx(0.3125)
    assert analytic.expected_rounds(10, 4) == pytest.approx(1.454545, rel=1e-5)
    assert analytic.tie_prob(683) == 0.0


def test_golden_vectors_reproduce(oracle_vectors):
    for c in oracle_vectors["states"][::3]:
        res = oracle.run_trials(c["N"], c["F"], c["faulty"], seed=c["seed"], trial_begin=c["trial"],
                                trial_count=1, k_max=c["k_max"], initial_values=c["init"], want_states=True)
        assert res.states == [decode_state(e) for e in c["states"]]
    for h in oracle_vectors["hists"]:
        if h["N"] * h["trial_count"] > 2_000_000:
            continue
        res = oracle.run_trials(h["N"], h["F"], [i < h["F"] for i in range(h["N"])], seed=h["seed"],
                                trial_begin=h["trial_begin"], trial_count=h["trial_count"], k_max=h["k_max"])
        assert {str(i): int(v) for i, v in enumerate(res.hist) if v} == h["hist_nonzero"]


# ------------------------------------------------- random delivery model
@pytest.mark.parametrize("m,q", [(10, 6), (100, 60), (100, 30), (1024, 683), (64, 64), (200, 1), (37, 0)])
def test_delivery_mask_exact_size_and_uniform(m, q):
    """Each receiver-phase tallies exactly q = N-F distinct live senders, and
    every sender is included with probability q/m (chi-square)."""
    from scipy import stats

    reps = 400 if m > 500 else 2000
    cnt = np.zeros(m)
    for node in range(reps):
        D = oracle.delivery_mask(0xABCDEF, 7, node, 3, node & 1, m, q)
        bits = np.array([(D[i >> 6] >> (i & 63)) & 1 for i in range(m)])
        assert bits.sum() == q
        if m % 64:
            assert D[-1] >> (m % 64) == 0
        cnt += bits
    if 0 < q < m:
        exp = np.full(m, reps * q / m)
        p = stats.chisquare(cnt, exp).pvalue
        assert p > 0.01, p


@pytest.mark.parametrize("m,q", [(7, 3), (10, 6), (8, 2), (16, 2), (16, 14)])
def test_delivery_subset_law_is_uniform(m, q):
    """Joint law, not only the marginals: every q-subset of the m senders is
    equally likely (chi-square over all C(m, q) subsets), Floyd sampler."""
    from math import comb

    from scipy import stats

    n = comb(m, q)
    reps = 40 * n
    cnt = {}
    for i in range(reps):
        D = oracle.delivery_mask(0x5EED, i // 7, i % 7, 1 + (i & 1), (i >> 1) & 1, m, q)
        cnt[D[0]] = cnt.get(D[0], 0) + 1
    assert len(cnt) == n and all(bin(k).count("1") == q for k in cnt)
    assert stats.chisquare(list(cnt.values())).pvalue > 0.01


def test_bernoulli_sampler_law_is_uniform():
    """Bernoulli + fix-up sampler (k >= 64): exact size, uniform marginals, and
    pairwise inclusion P(i, j in S) = q(q-1)/(m(m-1)) for every pair (a
    non-uniform subset law with uniform marginals would show up in the pair
    counts), chi-square p > 0.01."""
    from scipy import stats

    m, q, reps = 200, 72, 6000                      # k = 72 >= 64, 72 * 8 > 200: Bernoulli with p = 6/16
    assert oracle.delivery_bernoulli(m, q) == (6, 8)
    inc = np.zeros(m)
    pair = np.zeros(m // 2)                         # disjoint pairs (2i, 2i+1)
    for t in range(reps):
        D = oracle.delivery_mask(0xB0B, t, t % 13, 1 + t % 3, t & 1, m, q)
        bits = np.array([(D[i >> 6] >> (i & 63)) & 1 for i in range(m)])
        assert bits.sum() == q
        inc += bits
        pair += bits[0::2] & bits[1::2]
    assert stats.chisquare(inc, np.full(m, reps * q / m)).pvalue > 0.01
    p2 = q * (q - 1) / (m * (m - 1))
    z = (pair.sum() - reps * (m // 2) * p2) / np.sqrt(reps * (m // 2) * p2 * (1 - p2))
    assert abs(z) < 3


def test_delivery_sampler_choice():
    assert not oracle.delivery_bernoulli(1024, 1024 - 41)          # k = 41: Floyd
    assert oracle.delivery_bernoulli(1024, 683) == (11, 10)        # p = 11/16, 10-bit indices
    assert oracle.delivery_bernoulli(2100, 1400) == (11, 12)
    assert oracle.delivery_bernoulli(300, 100) == (6, 9)          # p = 3/8: 3 stream words per mask word
    assert not oracle.delivery_bernoulli(10, 6)                   # k = 4 < 64: Floyd
    assert not oracle.delivery_bernoulli(16, 2) and not oracle.delivery_bernoulli(64, 64)


def test_random_delivery_reduces_to_lockstep_at_f_equals_F():
    for N, F in [(10, 4), (64, 21), (130, 2), (5, 1)]:
        fl = [i < F for i in range(N)]
        a = oracle.run_trials(N, F, fl, seed=9, trial_count=3000, k_max=16, mode=oracle.MODE_RANDOM_DELIVERY)
        b = oracle.run_trials(N, F, fl, seed=9, trial_count=3000, k_max=16, mode=oracle.MODE_LOCKSTEP)
        np.testing.assert_array_equal(a.hist, b.hist)


def test_random_delivery_relative_majority_can_split():
    """With f < F the reference's relative-majority proposal (node.ts:63-69)
    lets different receivers propose different values, so split decisions
    appear: the agreement-violation counter is the model's report of it."""
    N, F = 1024, 341
    r = oracle.run_trials(N, F, [False] * N, seed=1, trial_count=60, k_max=16, mode=oracle.MODE_RANDOM_DELIVERY)
    assert r.hist.sum() - r.hist[-1] == 60
    assert r.hist[-1] > 0
    # with a strict-majority-sized fault bound the law is benign: f = F - 1 at N = 10, F = 2
    r = oracle.run_trials(10, 2, [True] + [False] * 9, seed=2, trial_count=20000, k_max=16,
                          mode=oracle.MODE_RANDOM_DELIVERY)
    assert r.hist[-1] == 0


# ------------------------------------------------- event-level mode
@pytest.mark.parametrize("N,F", [(5, 1), (10, 4), (12, 4), (9, 4), (10, 5), (16, 5)])
def test_event_mode_without_stop_equals_lockstep(N, F):
    """Exactly F faults and no mid-run /stop: every delivery order gives the
    lockstep outcome, per node and per histogram."""
    fl = [i < F for i in range(N)]
    a, ev = oracle.event_trials(N, F, fl, seed=21, trial_count=4000, k_max=16)
    b = oracle.run_trials(N, F, fl, seed=21, trial_count=4000, k_max=16)
    np.testing.assert_array_equal(a.hist, b.hist)
    assert ev > 0
    rng = np.random.default_rng(N)
    for t in range(20):
        init = [int(v) for v in rng.integers(0, 2, N)]
        sa, _ = oracle.event_trials(N, F, fl, seed=5, trial_begin=t, trial_count=1, k_max=16, initial_values=init,
                                    want_states=True)
        sb = oracle.run_trials(N, F, fl, seed=5, trial_begin=t, trial_count=1, k_max=16, initial_values=init,
                               want_states=True)
        assert sa.states == sb.states


def test_event_mode_stop_before_first_delivery_stalls():
    """A live node stopped before the first delivery: its round-1 proposals
    (already sent at /start) still arrive, so every running node completes the
    R-phase, but only N-F-1 nodes send votes -- no P-phase trigger can fire
    (node.ts:88); everyone sits at k = 1 (node.ts:172), undecided."""
    N, F = 10, 4
    ca = [None] * N
    ca[6] = 0
    r, ev = oracle.event_trials(N, F, [i < F for i in range(N)], seed=1, trial_count=1, k_max=16,
                                initial_values=[1] * N, crash_at=ca, want_states=True)
    live = r.states[F:]
    assert live[2]["killed"] and all(s["k"] == 1 and s["decided"] is False for s in live)
    assert r.hist[1] == 1 and ev == (N - F) * N + (N - F - 1) * N   # all round-1 messages, then nothing


def test_event_mode_stop_after_decision_is_harmless():
    N, F = 10, 4
    ca = [None] * N
    ca[7] = 10_000
    r, _ = oracle.event_trials(N, F, [i < F for i in range(N)], seed=1, trial_begin=7, trial_count=1, k_max=16,
                               initial_values=[1] * N, crash_at=ca, want_states=True)
    assert all(s["decided"] and s["x"] == 1 and s["k"] == 2 for s in r.states[F:])
