"""The matrix-core lockstep kernel (csrc/benor_mfma.h, BO_KERNEL_MFMA).

CPU: the host-side kernel choice (bo_kernel_for) -- which shapes go to the
matrix cores and which stay on the popcount / lane / random / event kernels.
GPU: bit-exact histograms against the oracle on every chunk count W = 2..16
(both tile parities), with fixed initial values and "?" inputs, partial
32-trial tiles and 64-bit trial offsets; equality with the popcount W kernel
(BENOR_NO_MFMA=1) over 10^6 trials; the network API (per-node state) on an
MFMA shape; and the init_q parity regression (the kernel choice depends on
the number of "?" initial values, which must be known before planning).
Deferral (KIND 1: m > 2F with ties; KIND 2: F < m <= 2F): trials that tie in
round 1 run rounds 2 and 3 in matrix-core continuation passes (x = the coins
of the tied round), and what still ties goes to the W kernel's trial-list mode
-- oracle histograms on both kinds and both m parities, several chunks of
deferred trials, and equality with the W kernel alone (9*10^6 trials at
N=128, F=0: ~6*10^5 trials reach round 2, ~4*10^4 round 3).
"""
import os

import numpy as np
import pytest

import benor
import oracle


def first_f(N, F):
    return [i < F for i in range(N)]


def mfma_shapes():
    """(N, F) with f = F crashed, m = N - F odd, m > 2F, 64 < m <= 1024: both
    tile parities (m - 64 (W-1) <= 32 or > 32) for every W, F at the bound and
    below it."""
    out = []
    for W in range(2, 17):
        for off in (1, 33, 63):
            m = 64 * (W - 1) + off
            for F in ((m - 1) // 2, (m - 1) // 5):
                out.append((m + F, F))
    return out


def plan(N, F, mfma=True, **kw):
    if mfma:
        os.environ.pop("BENOR_NO_MFMA", None)
    else:
        os.environ["BENOR_NO_MFMA"] = "1"
    try:
        return benor.TrialsPlan(N, F, **kw)
    finally:
        os.environ.pop("BENOR_NO_MFMA", None)


# ------------------------------------------------------------------ CPU
def test_kernel_choice():
    K = benor
    assert K.kernel_for(1024, 341) == K.BO_KERNEL_MFMA            # headline: m = 683 odd, m > 2F
    assert K.kernel_for(256, 85) == K.BO_KERNEL_MFMA              # configs[2]
    for N, F in mfma_shapes():
        assert K.kernel_for(N, F) == K.BO_KERNEL_MFMA, (N, F)
    assert K.kernel_for(1000, 300) == K.BO_KERNEL_MFMA            # m = 700 even: round 1 here, tied trials deferred
    assert K.kernel_for(1025, 512) == K.BO_KERNEL_MFMA            # m = 513 <= 2F: undecided trials deferred
    assert K.kernel_for(1024, 512) == K.BO_KERNEL_W               # m = F: no receiver can ever decide
    assert K.kernel_for(1537, 512) == K.BO_KERNEL_MFMA            # m = 1025: the big-network form
    assert K.kernel_for(4096, 1365) == K.BO_KERNEL_MFMA           # m = 2731
    assert K.kernel_for(4096, 2048) == K.BO_KERNEL_W              # m = F: never decides
    assert K.kernel_for(10, 4) == K.BO_KERNEL_MFMA_SMALL          # m <= 32, m > F: packed matrix-core kernel
    assert K.kernel_for(64, 21) == K.BO_KERNEL_LANE               # 32 < m <= 64
    assert K.kernel_for(96, 31) == K.BO_KERNEL_MFMA               # m = 65
    assert K.kernel_for(1024, 341, mode=K.BO_MODE_RANDOM_DELIVERY) == K.BO_KERNEL_RANDOM
    assert K.kernel_for(10, 4, mode=K.BO_MODE_EVENT) == K.BO_KERNEL_EVENT
    assert K.kernel_for(3, 3) == K.BO_KERNEL_NONE
    # fixed initial values: an odd number of "?" makes round 1's vote count even
    vals = [1] * 1024
    vals[500] = "?"
    assert K.kernel_for(1024, 341, initial_values=vals) == K.BO_KERNEL_MFMA   # M even: ties deferred
    vals[501] = "?"
    assert K.kernel_for(1024, 341, initial_values=vals) == K.BO_KERNEL_MFMA
    tied = [i % 2 for i in range(1024)]                                      # live 341..1023: 342 ones, 341 zeros
    assert K.kernel_for(1024, 341, initial_values=tied) == K.BO_KERNEL_MFMA
    tied[1023] = "?"                                                         # 341 / 341: every trial ties in round 1
    assert K.kernel_for(1024, 341, initial_values=tied) == K.BO_KERNEL_W
    os.environ["BENOR_NO_MFMA"] = "1"
    try:
        assert K.kernel_for(1024, 341) == K.BO_KERNEL_W
        assert K.kernel_for(4096, 1365) == K.BO_KERNEL_BLOCKED
    finally:
        os.environ.pop("BENOR_NO_MFMA", None)
    os.environ["BENOR_NO_MFMA_BIG"] = "1"
    try:
        assert K.kernel_for(1024, 341) == K.BO_KERNEL_MFMA
        assert K.kernel_for(2048, 682) == K.BO_KERNEL_W
        assert K.kernel_for(4096, 1365) == K.BO_KERNEL_BLOCKED
    finally:
        os.environ.pop("BENOR_NO_MFMA_BIG", None)


def test_kernel_choice_validates_like_plan_create():
    with pytest.raises(benor.Error, match="faultyList doesnt have F faulties"):
        benor.kernel_for(10, 4, [True] * 3 + [False] * 7)
    with pytest.raises(RuntimeError, match="k_max"):
        benor.kernel_for(10, 4, k_max=0)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("N,F", mfma_shapes())
def test_mfma_matches_oracle(N, F):
    seed = (N * 7919 + F) & 0xFFFF
    T = 977 + (N % 64)                       # partial last tile of 32 trials
    begin = (1 << 33) + N                    # 64-bit trial ids
    p = plan(N, F, seed=seed, k_max=8)
    assert p.kernel == benor.BO_KERNEL_MFMA
    got = p.run(begin, T)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=begin, trial_count=T, k_max=8)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
@pytest.mark.parametrize("N,F,q", [(300, 99, 2), (1024, 341, 10), (129, 40, 4), (97, 32, 0), (1001, 300, 6)])
def test_mfma_fixed_init_matches_oracle(N, F, q):
    rng = np.random.default_rng(N + q)
    vals = [int(v) for v in rng.integers(0, 2, N)]
    for j in rng.choice(np.arange(F, N), q, replace=False):
        vals[j] = "?"
    p = plan(N, F, seed=11, k_max=8, initial_values=vals)
    assert p.kernel == benor.BO_KERNEL_MFMA
    got = p.run(3, 333)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=11, trial_begin=3, trial_count=333, k_max=8,
                            initial_values=vals)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
@pytest.mark.parametrize("N,F", [(1024, 341), (256, 85), (97, 32), (1500, 477)])
def test_mfma_equals_popcount_kernel(N, F):
    a = plan(N, F, True, seed=99, k_max=16)
    b = plan(N, F, False, seed=99, k_max=16)
    assert a.kernel == benor.BO_KERNEL_MFMA and b.kernel == benor.BO_KERNEL_W
    np.testing.assert_array_equal(a.run(5, 1_000_003), b.run(5, 1_000_003))


@pytest.mark.gpu
def test_mfma_shape_network_api_per_node_state():
    """The per-node-state launch of an MFMA shape runs the W kernel; its
    states equal the oracle's (one trial)."""
    N, F = 256, 85
    rounds, st = benor.run_trial_states(N, F, first_f(N, F), seed=5, trial=42, k_max=8)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=5, trial_begin=42, trial_count=1, k_max=8, want_states=True)
    assert rounds == 1
    assert st == ref.states


@pytest.mark.gpu
@pytest.mark.parametrize("N,F,init", [
    (7, 0, [1, 0, "?", 1, 0, 1, 0]),                  # lane kernel: m = 7, one "?": round-1 M = 6 (ties)
    (11, 2, [1, 1, 0, "?", 0, 1, 0, 1, 1, 0, "?"]),    # m = 9, two "?" on live nodes
    (301, 100, None),                                 # W kernel: m = 201, one "?" below
])
def test_question_mark_parity_picks_the_right_kernel(N, F, init):
    if init is None:
        rng = np.random.default_rng(0)
        init = [int(v) for v in rng.integers(0, 2, N)]
        init[150] = "?"
    p = benor.TrialsPlan(N, F, seed=21, k_max=12, initial_values=init)
    got = p.run(0, 4000)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=21, trial_begin=0, trial_count=4000, k_max=12,
                            initial_values=init)
    np.testing.assert_array_equal(got, ref.hist)


def deferral_shapes():
    """(N, F, kind): KIND 1 (m > 2F, m even: ties) and KIND 2 (F < m <= 2F,
    both parities), across tile parities and chunk counts."""
    return [(100, 0, 1), (256, 0, 1), (700, 200, 1), (1024, 0, 1), (1000, 333, 1), (97, 31, 1),
            (129, 64, 2), (130, 64, 2), (300, 140, 2), (513, 256, 2), (1024, 500, 2), (1500, 700, 2)]


@pytest.mark.gpu
@pytest.mark.parametrize("N,F,kind", deferral_shapes())
def test_mfma_deferral_matches_oracle(N, F, kind):
    seed = (N * 31 + F) & 0xFFFF
    T = 1500 + (N % 97)
    begin = (1 << 34) + 17 * N
    p = plan(N, F, seed=seed, k_max=12)
    assert p.kernel == benor.BO_KERNEL_MFMA
    got = p.run(begin, T)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=begin, trial_count=T, k_max=12)
    np.testing.assert_array_equal(got, ref.hist)
    # even m at m > 2F defers exactly the round-1 ties (q(m) of the trials)
    assert got[3:6].sum() < T or (N - F) % 2 == 1


@pytest.mark.gpu
@pytest.mark.parametrize("N,F,q", [(300, 99, 1), (1024, 341, 3), (129, 40, 1), (500, 200, 5)])
def test_mfma_deferral_fixed_init_matches_oracle(N, F, q):
    """Fixed starts with an odd number of "?" inputs: round 1 has an even vote
    count; a tied start is planned on the W kernel."""
    rng = np.random.default_rng(N * 3 + q)
    vals = [int(v) for v in rng.integers(0, 2, N)]
    for j in rng.choice(np.arange(F, N), q, replace=False):
        vals[j] = "?"
    p = plan(N, F, seed=13, k_max=10, initial_values=vals)
    live = vals[F:]
    tie = live.count(0) == live.count(1)
    assert p.kernel == (benor.BO_KERNEL_W if tie else benor.BO_KERNEL_MFMA)
    got = p.run(7, 777)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=13, trial_begin=7, trial_count=777, k_max=10,
                            initial_values=vals)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
@pytest.mark.parametrize("k_max", [1, 2, 3])
@pytest.mark.parametrize("N,F", [(256, 0), (1000, 333), (300, 140), (2048, 0), (3000, 1400)])
def test_mfma_deferral_small_kmax_matches_oracle(N, F, k_max):
    """k_max 1..3 against the continuation passes: the host runs
    matrix-core rounds 2 .. min(3, k_max - 1) and leaves the rest to the
    popcount kernel, whose trials then reach k_max undecided.  KIND 1 and 2,
    small- and big-network forms."""
    seed = 0xC0FFEE ^ (N << 8) ^ k_max
    p = plan(N, F, seed=seed, k_max=k_max)
    assert p.kernel == benor.BO_KERNEL_MFMA
    begin, T = (1 << 33) + 3 * N, 3000 + N % 71
    got = p.run(begin, T)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=begin, trial_count=T, k_max=k_max)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
def test_mfma_deferral_two_chunks_matches_oracle():
    """One launch just above kDeferChunk (2^22) trials at a non-zero trial_begin:
    the second deferral chunk starts at trial_begin + 2^22."""
    N, F, seed = 100, 0, 99
    T, begin = (1 << 22) + 1001, (1 << 32) + 12345
    p = plan(N, F, seed=seed, k_max=8)
    assert p.kernel == benor.BO_KERNEL_MFMA
    got = p.run(begin, T)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=begin, trial_count=T, k_max=8,
                            threads=min(16, os.cpu_count() or 1))
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
@pytest.mark.parametrize("N,F,T", [(128, 0, 9_000_001), (1024, 0, 1_000_003), (600, 250, 2_000_001), (257, 127, 5_000_000)])
def test_mfma_deferral_equals_popcount_kernel(N, F, T):
    """Over several deferral chunks (kDeferChunk = 2^22 trials): the same
    histogram as the popcount kernels alone, and a split launch sums to it."""
    a = plan(N, F, True, seed=5, k_max=24)
    b = plan(N, F, False, seed=5, k_max=24)
    assert a.kernel == benor.BO_KERNEL_MFMA and b.kernel != benor.BO_KERNEL_MFMA
    ha = a.run(11, T)
    np.testing.assert_array_equal(ha, b.run(11, T))
    cut = T // 3 + 5
    np.testing.assert_array_equal(ha, a.run(11, cut) + a.run(11 + cut, T - cut))


def big_shapes():
    """1024 < m <= 4096 (W = 17..64, the big-network form): every KIND, both
    m parities, tile-pair parity (odd ceil(m/32)), W kernel (W <= 32) and
    blocked kernel (W > 32) for the deferred trials."""
    return [(1100, 0), (1537, 512), (1600, 500), (2047, 1), (2048, 682), (2080, 1000), (2731, 0),
            (3000, 999), (3333, 1500), (4096, 1365), (4096, 0), (4000, 1900), (4095, 1), (2049, 1024)]


@pytest.mark.gpu
@pytest.mark.parametrize("N,F", big_shapes())
def test_mfma_big_matches_oracle(N, F):
    seed = (N * 131 + F) & 0xFFFF
    T = 333 + (N % 61)
    begin = (1 << 35) + N
    p = plan(N, F, seed=seed, k_max=10)
    assert p.kernel == benor.BO_KERNEL_MFMA
    got = p.run(begin, T)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=begin, trial_count=T, k_max=10)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
@pytest.mark.parametrize("form", [("wave", None), ("coop", "4"), ("coop", "8")])
@pytest.mark.parametrize("N,F", [(1100, 0), (2049, 1024), (2080, 1000), (3333, 1500), (4096, 1365), (4096, 0)])
def test_mfma_big_forms_match_oracle(N, F, form):
    """Both big-network forms -- per-wave (benor_mfma_big.hip) and
    workgroup-cooperative with 4 or 8 waves (benor_mfma_coop.hip) -- forced by
    environment on every KIND, round 1 and the continuation passes, against
    the oracle (the default picks one form per W)."""
    seed = (N * 7 + F) & 0xFFFF
    T, begin = 700 + N % 37, (1 << 34) + F
    keys = {"BENOR_BIG_FORM": form[0]}
    if form[1]:
        keys["BENOR_COOP_BW"] = form[1]
    old = {k: os.environ.get(k) for k in keys}
    os.environ.update(keys)
    try:
        p = plan(N, F, seed=seed, k_max=10)
        assert p.kernel == benor.BO_KERNEL_MFMA
        got = p.run(begin, T)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    ref = oracle.run_trials(N, F, first_f(N, F), seed=seed, trial_begin=begin, trial_count=T, k_max=10)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
@pytest.mark.parametrize("N,F,T", [(2048, 0, 300_000), (4096, 1365, 200_001), (3000, 1400, 250_000), (1500, 200, 400_000)])
def test_mfma_big_equals_popcount_kernels(N, F, T):
    a = plan(N, F, True, seed=17, k_max=16)
    os.environ["BENOR_NO_MFMA_BIG"] = "1"
    try:
        b = benor.TrialsPlan(N, F, seed=17, k_max=16)
    finally:
        os.environ.pop("BENOR_NO_MFMA_BIG", None)
    assert a.kernel == benor.BO_KERNEL_MFMA and b.kernel != benor.BO_KERNEL_MFMA
    np.testing.assert_array_equal(a.run(3, T), b.run(3, T))


@pytest.mark.gpu
@pytest.mark.parametrize("N,F", [(3000, 900), (4096, 1900)])
def test_mfma_coop_two_chunks_equals_popcount_kernels(N, F):
    """The cooperative big-network form over two deferral chunks (kDeferChunk =
    2^22 trials) from a 64-bit trial_begin: per-workgroup deferral segments,
    both continuation passes and the popcount remainder of each chunk give the
    popcount kernels' histogram (KIND 1 at W = 33; KIND 2 at W = 35)."""
    T, begin = (1 << 22) + 777, (1 << 33) + 5
    a = plan(N, F, True, seed=41, k_max=12)
    os.environ["BENOR_NO_MFMA_BIG"] = "1"
    try:
        b = benor.TrialsPlan(N, F, seed=41, k_max=12)
    finally:
        os.environ.pop("BENOR_NO_MFMA_BIG", None)
    assert a.kernel == benor.BO_KERNEL_MFMA and b.kernel != benor.BO_KERNEL_MFMA
    np.testing.assert_array_equal(a.run(begin, T), b.run(begin, T))


@pytest.mark.gpu
@pytest.mark.parametrize("N,F,q", [(2000, 600, 1), (4096, 1000, 2), (1500, 700, 3)])
def test_mfma_big_fixed_init_matches_oracle(N, F, q):
    rng = np.random.default_rng(N + 7 * q)
    vals = [int(v) for v in rng.integers(0, 2, N)]
    for j in rng.choice(np.arange(F, N), q, replace=False):
        vals[j] = "?"
    p = plan(N, F, seed=23, k_max=8, initial_values=vals)
    got = p.run(1, 200)
    ref = oracle.run_trials(N, F, first_f(N, F), seed=23, trial_begin=1, trial_count=200, k_max=8,
                            initial_values=vals)
    np.testing.assert_array_equal(got, ref.hist)


@pytest.mark.gpu
def test_mfma_peak_probe():
    peak = benor.mfma_peak(3)
    assert 1e15 < peak < 6e15                # dense e2m1 spec: 5e15 multiply-adds/s


# ------------------------------------------------- deferral segment invariant
def seg_cap_of(trials, units):
    """The runtime's segment sizing (benor_runtime.cpp plan_launch_impl):
    ceil(groups / units) 32-trial groups per owner."""
    groups = (trials + 31) // 32
    return (groups + units - 1) // units * 32


@pytest.mark.parametrize("trials", [1, 31, 32, 33, 1000, 4096 * 32 + 5, (1 << 22)])
@pytest.mark.parametrize("units", [1, 3, 64, 1024, 2048 * 4, 1 << 16])
def test_deferral_segment_sizing_covers_every_owner(trials, units):
    """Owner w of a launch (wave, or workgroup of the cooperative form) walks
    the 32-trial groups w, w + units, ... (grid-stride), and every trial of a
    group can defer: the segment must hold 32 x the most groups an owner gets."""
    groups = (trials + 31) // 32
    most = max(len(range(w, groups, units)) for w in range(min(units, groups))) if groups else 0
    assert 32 * most <= seg_cap_of(trials, units)


class _env:
    """Set environment variables for a block (None = leave unset)."""
    def __init__(self, **kv):
        self.kv = {k: v for k, v in kv.items() if v is not None}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.gpu
@pytest.mark.parametrize("N,F,form", [(256, 0, None), (300, 120, None), (3000, 900, "coop"), (2048, 0, "wave")])
def test_deferral_overflow_is_reported(N, F, form):
    """A segment capacity below the sizing rule (BENOR_TEST_DEFER_SEG_CAP=1)
    makes owners drop deferred trials: bo_plan_run must fail with
    BO_ERR_INTERNAL instead of returning an incomplete histogram, and the
    next run at the normal capacity is clean and matches the popcount kernel."""
    T = 200_000 if N <= 300 else 40_000
    with _env(BENOR_BIG_FORM=form):
        p = plan(N, F, seed=3, k_max=12)
        assert p.kernel == benor.BO_KERNEL_MFMA
        with _env(BENOR_TEST_DEFER_SEG_CAP="1"):
            with pytest.raises(RuntimeError, match="libbenor error 9"):
                p.run(0, T)
        got = p.run(0, T)
        p.check()
    with _env(BENOR_NO_MFMA="1", BENOR_NO_MFMA_BIG="1"):
        ref = benor.TrialsPlan(N, F, seed=3, k_max=12).run(0, T)
    np.testing.assert_array_equal(got, ref)
