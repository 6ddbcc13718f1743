"""Differential fuzzing of the GPU kernels against the CPU oracle through the
C ABI: seeded random network shapes (N up to 4096, F including F >= N/2),
arbitrary fault placements, random or fixed initial values (with "?"
entries, so the first round's binary vote count M differs from m), and
small / large round caps.  Covers every lockstep kernel variant (packed,
W kernel, odd / even / "every receiver decides" decision paths, blocked) and
the random-delivery and event-level modes.  At these trial counts a wave
holds about one trial, so the W kernel's interleaved round 1 is covered by
test_gpu_parity.py::test_interleaved_round1_matches_oracle instead.
Histograms must be bit-identical."""
import numpy as np
import pytest

import benor
import oracle

pytestmark = pytest.mark.gpu

RD, EV = benor.BO_MODE_RANDOM_DELIVERY, benor.BO_MODE_EVENT


def _shape(rng, n_lo, n_hi):
    N = int(rng.integers(n_lo, n_hi + 1))
    F = int(rng.integers(0, N // 2 + 2)) if N > 1 else 0
    F = min(F, N)
    return N, F


def _placement(rng, N, f):
    fl = [False] * N
    for i in rng.choice(N, f, replace=False):
        fl[int(i)] = True
    return fl


def _init(rng, N, fixed):
    if not fixed:
        return None
    vals = rng.choice([0, 1, 2], size=N, p=[0.45, 0.45, 0.10])
    return ["?" if v == 2 else int(v) for v in vals]


def _trials_for(m):
    return 3000 if m <= 64 else (600 if m <= 512 else (150 if m <= 2048 else 40))


@pytest.mark.parametrize("case", range(120))
def test_lockstep_fuzz(case):
    rng = np.random.default_rng(1000 + case)
    lo, hi = [(1, 40), (33, 300), (300, 1100), (1000, 2100), (2000, 4096)][case % 5]
    N, F = _shape(rng, lo, hi)
    fl = _placement(rng, N, F)
    init = _init(rng, N, fixed=bool(case % 3 == 0))
    k_max = int(rng.choice([3, 12, 40]))
    seed = int(rng.integers(0, 2**63))
    T = _trials_for(N - F)
    plan = benor.TrialsPlan(N, F, fl, seed=seed, k_max=k_max, initial_values=init)
    got = plan.run(12345, T)
    ref = oracle.run_trials(N, F, fl, seed=seed, trial_begin=12345, trial_count=T, k_max=k_max,
                            initial_values=init).hist
    np.testing.assert_array_equal(got, ref, err_msg=f"N={N} F={F} k_max={k_max} init={'fixed' if init else 'random'}")


@pytest.mark.parametrize("case", range(40))
def test_random_delivery_fuzz(case):
    rng = np.random.default_rng(5000 + case)
    N, F = _shape(rng, 4, 700 if case % 3 else 2200)
    f = int(rng.integers(0, F + 1))
    fl = _placement(rng, N, f)
    init = _init(rng, N, fixed=bool(case % 4 == 0))
    k_max = int(rng.choice([4, 16]))
    seed = int(rng.integers(0, 2**63))
    m = N - f
    T = 400 if m <= 64 else (40 if m <= 512 else 6)
    got = benor.TrialsPlan(N, F, fl, seed=seed, k_max=k_max, initial_values=init, mode=RD).run(77, T)
    ref = oracle.run_trials(N, F, fl, seed=seed, trial_begin=77, trial_count=T, k_max=k_max, initial_values=init,
                            mode=oracle.MODE_RANDOM_DELIVERY).hist
    np.testing.assert_array_equal(got, ref, err_msg=f"N={N} F={F} f={f}")


@pytest.mark.parametrize("case", range(24))
def test_event_fuzz(case):
    rng = np.random.default_rng(9000 + case)
    N = int(rng.integers(2, 33))
    F = int(rng.integers(0, N // 2 + 1))
    fl = _placement(rng, N, F)
    init = _init(rng, N, fixed=bool(case % 2))
    seed = int(rng.integers(0, 2**63))
    cc = int(rng.integers(0, 3))
    cw = int(rng.integers(1, 4 * N * N))
    T = 300
    got = benor.TrialsPlan(N, F, fl, seed=seed, k_max=12, initial_values=init, mode=EV, crash_count=cc,
                           crash_window=cw).run(3, T)
    ref, _ = oracle.event_trials(N, F, fl, seed=seed, trial_begin=3, trial_count=T, k_max=12, initial_values=init,
                                 crash_count=cc, crash_window=cw)
    np.testing.assert_array_equal(got, ref.hist, err_msg=f"N={N} F={F} crash {cc}/{cw}")
