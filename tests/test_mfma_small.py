"""The packed matrix-core kernel for small networks (csrc/benor_mfma_small.h,
BO_KERNEL_MFMA_SMALL): 2 <= m <= 32 live nodes, m > F, no "?" initial value;
min(32/m, 8) trials per lane half, block-diagonal e2m1 products.

CPU: which shapes it takes.  GPU: bit-exact histograms against the oracle
(oracle/benor_oracle.c bit-plane restatement of node.ts:43-163) for every m in
2..32 at F on both sides of m/2, random and fixed initial values, k_max 1..4
(the matrix-core rounds, their list hand-offs and the lane path), partial
batches and 64-bit trial offsets; equality with the lane kernel
(BENOR_NO_MFMA=1) over 10^6-10^7 trials at BASELINE configs[1] (N=10, F=4)
and configs[0]'s shape (N=5, F=1); split-launch invariance; the lane
kernel's own parity on the shapes the packed kernel took from it.
"""
import os

import numpy as np
import pytest

import benor
import oracle


@pytest.fixture(autouse=True)
def packed_for_every_launch(monkeypatch):
    """Launches shorter than kSmallMinTrials run the lane kernel; these tests
    pin the packed kernel itself at every trial count."""
    monkeypatch.setenv("BENOR_SMALL_MIN_TRIALS", "0")


def first_f(N, F):
    return [i < F for i in range(N)]


def plan(N, F, mfma=True, **kw):
    if mfma:
        os.environ.pop("BENOR_NO_MFMA", None)
    else:
        os.environ["BENOR_NO_MFMA"] = "1"
    try:
        return benor.TrialsPlan(N, F, **kw)
    finally:
        os.environ.pop("BENOR_NO_MFMA", None)


def test_kernel_choice_small():
    K = benor
    assert K.kernel_for(10, 4) == K.BO_KERNEL_MFMA_SMALL          # configs[1]: m = 6 > F
    assert K.kernel_for(5, 1) == K.BO_KERNEL_MFMA_SMALL           # configs[0] shape: m = 4
    assert K.kernel_for(10, 5) == K.BO_KERNEL_LANE                # F > N/2 case: m = 5 <= F, never decides
    assert K.kernel_for(33, 1) == K.BO_KERNEL_MFMA_SMALL          # m = 32
    assert K.kernel_for(34, 1) == K.BO_KERNEL_LANE                # m = 33
    assert K.kernel_for(2, 0) == K.BO_KERNEL_MFMA_SMALL           # m = 2
    assert K.kernel_for(1, 0) == K.BO_KERNEL_LANE                 # m = 1
    assert K.kernel_for(10, 4, initial_values=[0] * 4 + [1, "?", 0, 1, 1, 0]) == K.BO_KERNEL_LANE   # "?" input
    assert K.kernel_for(10, 4, initial_values=[0] * 4 + [1, 1, 0, 1, 1, 0]) == K.BO_KERNEL_MFMA_SMALL
    assert K.kernel_for(10, 4, mode=K.BO_MODE_RANDOM_DELIVERY) == K.BO_KERNEL_RANDOM
    os.environ["BENOR_NO_MFMA"] = "1"
    try:
        assert K.kernel_for(10, 4) == K.BO_KERNEL_LANE
    finally:
        os.environ.pop("BENOR_NO_MFMA", None)


def small_shapes():
    out = []
    for m in range(2, 33):
        for F in sorted({0, (m - 1) // 2, m - 1}):
            out.append((m + F, F))
    return out




@pytest.mark.gpu
@pytest.mark.parametrize("N,F", small_shapes())
def test_mfma_small_matches_oracle(N, F):
    m = N - F
    seed = (m * 7919 + F) & 0xFFFFFFFF
    k_max = 16
    p = plan(N, F, seed=seed, k_max=k_max)
    assert p.kernel == benor.BO_KERNEL_MFMA_SMALL
    S = min(32 // m, 8)
    T = 3 * 64 * S * 4 + 77 + m                  # several batches per wave, a partial one
    begin = (1 << 33) + 5 * N
    got = p.run(begin, T)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=begin, trial_count=T, k_max=k_max)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
@pytest.mark.parametrize("k_max", [1, 2, 3, 4])
@pytest.mark.parametrize("N,F", [(10, 4), (5, 1), (8, 0), (20, 8), (34, 2), (14, 2)])
def test_mfma_small_kmax_matches_oracle(N, F, k_max):
    """k_max below, at and above the matrix-core rounds (3): ties hand over to
    the round lists or the lane path, which runs the trial to k_max."""
    seed = 0xA11CE + 131 * N + k_max
    p = plan(N, F, seed=seed, k_max=k_max)
    assert p.kernel == benor.BO_KERNEL_MFMA_SMALL
    got = p.run(17, 40_000)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=17, trial_count=40_000, k_max=k_max)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
@pytest.mark.parametrize("N,F,vals", [
    (10, 4, [0] * 4 + [1, 1, 0, 1, 1, 0]),        # 3 vs 3: every trial ties in round 1
    (10, 4, [0] * 4 + [1, 1, 1, 1, 1, 0]),        # decides in round 1
    (5, 1, [1, 1, 1, 0, 0]),                       # benorconsensus.test.ts:179-223 "Simple Majority"
    (7, 1, [0, 1, 0, 1, 0, 1, 1]),
    (32, 0, [i % 2 for i in range(32)]),           # m = 32 tie
])
def test_mfma_small_fixed_init_matches_oracle(N, F, vals):
    p = plan(N, F, seed=5, k_max=12, initial_values=vals)
    assert p.kernel == benor.BO_KERNEL_MFMA_SMALL
    got = p.run(3, 25_000)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=5, trial_begin=3, trial_count=25_000, k_max=12,
                            initial_values=vals)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
def test_mfma_small_random_fault_placement():
    rng = np.random.default_rng(4)
    for N in (6, 11, 17, 30, 40):
        F = int(rng.integers(0, N // 2 + 1))
        faulty = [False] * N
        for i in rng.choice(N, F, replace=False):
            faulty[i] = True
        if N - F > 32:
            continue
        p = benor.TrialsPlan(N, F, faulty, seed=N, k_max=10)
        assert p.kernel == benor.BO_KERNEL_MFMA_SMALL
        got = p.run(0, 30_000)
        ref = oracle.run_trials(N, F, faulty, seed=N, trial_begin=0, trial_count=30_000, k_max=10)
        np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
@pytest.mark.parametrize("N,F,T,k_max", [
    (10, 4, 1_000_000, 16),               # configs[1]: 3 full strides of 1024 waves + 53 batches
    (10, 4, 3 * 1024 * 320 + 64 * 1024, 16),
    (10, 4, 3 * 1024 * 320 + 64 * 1024 + 1, 16),
    (32, 0, 2 * 1024 * 64 + 1_000, 4),   # S = 1
    (20, 4, 1024 * 128 + 4_097, 2),      # S = 2, k_max below the matrix-core rounds
    (9, 4, 1024 * 384 + 77, 16),         # m = 5, F = 4 (S = 6)
])
def test_mfma_small_full_launch_matches_oracle(N, F, T, k_max):
    """Launches of >= 1024 batches (the full grid on a 256-CU MI355X, several
    fresh strides per wave and a short last one), their histogram against the
    oracle itself rather than the lane kernel."""
    seed = 0x5151 + 97 * N + T
    p = plan(N, F, seed=seed, k_max=k_max)
    assert p.kernel == benor.BO_KERNEL_MFMA_SMALL
    begin = (1 << 32) - 1000
    got = p.run(begin, T)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=begin, trial_count=T, k_max=k_max)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
@pytest.mark.parametrize("N,F,T", [(10, 4, 1_000_000), (5, 1, 2_000_003), (10, 4, 10_000_000), (16, 7, 3_000_000)])
def test_mfma_small_equals_lane_kernel(N, F, T):
    """BASELINE configs[1] at its 10^6 trials and beyond: the histogram of the
    lane kernel alone, and a split launch sums to it."""
    a = plan(N, F, True, seed=0x243F6A8885A308D3, k_max=16)
    b = plan(N, F, False, seed=0x243F6A8885A308D3, k_max=16)
    assert a.kernel == benor.BO_KERNEL_MFMA_SMALL and b.kernel == benor.BO_KERNEL_LANE
    ha = a.run(0, T)
    np.testing.assert_array_equal(ha, b.run(0, T))
    cut = T // 3 + 11
    np.testing.assert_array_equal(ha, a.run(0, cut) + a.run(cut, T - cut))


@pytest.mark.gpu
@pytest.mark.parametrize("T", [300_000, 1_000_000])
def test_short_launch_crossover_same_histogram(monkeypatch, T):
    """Under the default crossover (5*10^5 trials) a 3*10^5-trial launch of
    configs[1] runs on the lane kernel and a 10^6 one (configs[1]'s own
    count) on the packed kernel; both equal the other kernel's histogram."""
    monkeypatch.delenv("BENOR_SMALL_MIN_TRIALS")
    p = plan(10, 4, seed=99, k_max=16)
    h = p.run(7, T)
    monkeypatch.setenv("BENOR_SMALL_MIN_TRIALS", "0" if T < 500_000 else str(1 << 40))
    np.testing.assert_array_equal(h, p.run(7, T))


@pytest.mark.gpu
@pytest.mark.parametrize("N,F", [(10, 4), (5, 1), (33, 1), (9, 0)])
def test_lane_kernel_on_packed_shapes_matches_oracle(N, F):
    """The lane kernel keeps serving these shapes' per-node state launches and
    BENOR_NO_MFMA runs: its batch path stays oracle-checked on them."""
    p = plan(N, F, False, seed=77, k_max=16)
    assert p.kernel == benor.BO_KERNEL_LANE
    got = p.run(9, 50_000)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=77, trial_begin=9, trial_count=50_000, k_max=16)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
def test_packed_shape_network_api_states():
    """The network API's one-trial state launch of a packed shape runs the
    lane kernel: benorconsensus.test.ts "Simple Majority" states."""
    benor.launchNetwork(5, 1, [1, 1, 1, 0, 0], [False, False, False, False, True])
    benor.startConsensus(5, seed=3, sync=True)
    st = benor.getNodesState(5)
    assert all(s["decided"] and s["x"] == 1 and s["k"] == 2 for s in st[:4])
