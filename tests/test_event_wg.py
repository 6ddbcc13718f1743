"""The workgroup-batched event kernel (csrc/benor_event_live.hip, r06) against
oracle (iii), oracle/benor_oracle.c event_trial().

It runs every live run (the default startConsensus) and every network start
with a /stop schedule, one trial per workgroup: a control wave plus 1, 3, 7 or
15 event waves that resolve a batch of deliveries at once, cut at its first
pick conflict and at its first quorum (node.ts:52, :88).  Checked here:

* histograms of many trials against the oracle (BENOR_EVENT_FORM=wg routes
  batch event plans to it), with no stop, explicit and random /stop
  schedules, at N from 1 to 1024, every wave count, both pool forms (LDS for
  N <= 78, HBM above), and its one-wave forms (the register kernel at
  N <= 16, the LDS micro-batch kernel at N <= 64; BENOR_EVENT_FORM=wave
  puts the small N on the latter);
* live runs' GET /getState snapshots (bo_get_states): each equals oracle (iii)
  truncated at the delivery count the snapshot reports, with the killed flag
  of every /stop already posted (node.ts:191-194);
* per-node states of scheduled runs (the network API) at N = 5 .. 4096.
"""
import time

import numpy as np
import pytest

import benor
import oracle

pytestmark = pytest.mark.gpu


def first_f(N, F):
    return [i < F for i in range(N)]


def wg_hist(monkeypatch, N, F, *, waves=None, seed, trials, k_max=16, init=None, crash_at=None, crash_count=0,
            crash_window=0, form="wg"):
    monkeypatch.setenv("BENOR_EVENT_FORM", form)
    if waves:
        monkeypatch.setenv("BENOR_LIVE_WAVES", str(waves))
    plan = benor.TrialsPlan(N, F, first_f(N, F), seed=seed, k_max=k_max, initial_values=init,
                            mode=benor.BO_MODE_EVENT, crash_at=crash_at, crash_count=crash_count,
                            crash_window=crash_window)
    h = plan.run(3, trials)
    monkeypatch.delenv("BENOR_EVENT_FORM")
    monkeypatch.delenv("BENOR_LIVE_WAVES", raising=False)
    return h


def ref_hist(N, F, *, seed, trials, k_max=16, init=None, crash_at=None, crash_count=0, crash_window=0):
    res, _ = oracle.event_trials(N, F, first_f(N, F), seed=seed, trial_begin=3, trial_count=trials, k_max=k_max,
                                 initial_values=init, crash_at=crash_at, crash_count=crash_count,
                                 crash_window=crash_window)
    return res.hist


@pytest.mark.parametrize("N,F,trials", [
    (1, 0, 64), (3, 1, 400), (5, 1, 400), (10, 4, 400), (10, 5, 200), (16, 5, 300), (31, 10, 200),
    (32, 10, 200), (64, 21, 100), (78, 26, 60), (79, 26, 60), (100, 33, 40), (256, 85, 12), (300, 71, 8),
    (1024, 341, 3),
])
def test_histograms_match_oracle(monkeypatch, N, F, trials):
    """Random initial values (ties and coins at even m), no /stop."""
    seed = 0xE1 + N
    got = wg_hist(monkeypatch, N, F, seed=seed, trials=trials)
    np.testing.assert_array_equal(got, ref_hist(N, F, seed=seed, trials=trials))


@pytest.mark.parametrize("waves", [1, 3, 7, 15])
@pytest.mark.parametrize("N,F", [(20, 6), (100, 33), (160, 80)])
def test_every_wave_count(monkeypatch, waves, N, F):
    """Each workgroup shape, with the pool in LDS (N = 20) and in HBM (N = 100,
    160); N = 160, F = 80 never decides (m <= 2F): k_max rounds."""
    seed, trials = 0xA0 + waves, 24
    got = wg_hist(monkeypatch, N, F, waves=waves, seed=seed, trials=trials)
    np.testing.assert_array_equal(got, ref_hist(N, F, seed=seed, trials=trials))


@pytest.mark.parametrize("N,F,stops", [
    (10, 4, {4: 0, 7: 13}), (10, 5, {6: 40}), (64, 21, {30: 1000, 40: 2500}),
    (300, 71, {100: 30_000}), (1024, 341, {500: 200_000, 900: 699_000}),
])
def test_explicit_stop_schedules(monkeypatch, N, F, stops):
    """GET /stop at fixed delivery counts (node.ts:191-194): inside round 1, at
    its end and in round 2; a stop at delivery 0."""
    crash = [stops.get(i) for i in range(N)]
    seed, trials = 0x5C + N, 6 if N < 1000 else 2
    got = wg_hist(monkeypatch, N, F, seed=seed, trials=trials, crash_at=crash)
    np.testing.assert_array_equal(got, ref_hist(N, F, seed=seed, trials=trials, crash_at=crash))


@pytest.mark.parametrize("N,F,count,window,trials", [
    (10, 4, 1, 80, 300), (10, 4, 3, 200, 300), (40, 13, 2, 3000, 60), (300, 71, 4, 60_000, 6),
    (1024, 341, 3, 1_500_000, 2),
])
def test_random_stop_schedules(monkeypatch, N, F, count, window, trials):
    """crash_count live nodes stopped at uniform delivery counts in [0, window),
    drawn per trial (Philox stream 4, Floyd), as oracle (iii)."""
    seed = 0xC7 + N
    got = wg_hist(monkeypatch, N, F, seed=seed, trials=trials, crash_count=count, crash_window=window)
    np.testing.assert_array_equal(got, ref_hist(N, F, seed=seed, trials=trials, crash_count=count,
                                                crash_window=window))


@pytest.mark.parametrize("N,F,stops", [
    (1, 0, {}), (3, 1, {}), (10, 4, {4: 0, 7: 13}), (10, 5, {}), (16, 5, {3: 200}), (15, 7, {}), (16, 8, {0: 50}),
])
def test_wave_form_below_the_register_form(monkeypatch, N, F, stops):
    """N <= 16 runs on the register kernel (the pool in VGPRs, one event per
    step); BENOR_EVENT_FORM=wave runs the same plans on the LDS micro-batch
    kernel that N = 23 .. 64 use.  Both against the oracle."""
    crash = [stops.get(i) for i in range(N)] if stops else None
    seed, trials = 0x3B + N, 120
    want = ref_hist(N, F, seed=seed, trials=trials, crash_at=crash)
    for form in ("wg", "wave"):
        got = wg_hist(monkeypatch, N, F, seed=seed, trials=trials, crash_at=crash, form=form)
        np.testing.assert_array_equal(got, want, err_msg=form)


def test_fixed_ties_and_question_marks(monkeypatch):
    """Fixed starts: a tied round 1 (every node takes its coin), '?' values."""
    N, F = 21, 6
    init = [0] * F + [1, 0] * 7 + ["?"]
    got = wg_hist(monkeypatch, N, F, seed=0x7E, trials=100, init=init)
    np.testing.assert_array_equal(got, ref_hist(N, F, seed=0x7E, trials=100, init=init))


# ------------------------------------------------------------------ live snapshots
def shape(N, F, live_init):
    return [i < F for i in range(N)], [0] * F + list(live_init)


def ties(m):
    return [1] * (m // 2) + [0] * (m // 2) + ["?"] * (m % 2)


def check_snapshots(N, F, faulty, init, seed, k_max, snaps, events, posted_before):
    """Every snapshot (states, e) equals oracle (iii) truncated at e, with the
    stops landed at `events` replayed and the killed flag of every stop posted
    before the snapshot was requested."""
    sched = [None if v is None else v for v in events]
    mid = [j for j, (_, e) in enumerate(snaps) if e is not None]
    if len(mid) > 12:                                  # the oracle replays e deliveries per check
        mid = sorted({mid[round(i * (len(mid) - 1) / 11)] for i in range(12)})
    checked = 0
    for j in mid:
        states, e = snaps[j]
        want, _ = oracle.event_states_at(N, F, faulty, e, seed=seed, k_max=k_max, initial_values=init,
                                         crash_at=sched)
        for i in posted_before[j]:
            want[i] = dict(want[i], killed=True)
        assert states == want, (j, e)
        checked += 1
    return checked


@pytest.mark.parametrize("N,F,k_max", [(1024, 341, 16), (10, 5, 64), (100, 50, 64), (4096, 1365, 16)])
def test_live_snapshots_match_truncated_oracle(N, F, k_max):
    """GET /getState during a live run answers at once with the
    running network's states (node.ts:197-199).  Snapshots are taken as fast as
    the caller asks until the run ends; each equals oracle (iii) truncated at
    its delivery count.  At N = 1024 a node is stopped half-way through: the
    snapshots after the request carry its killed flag before and after the
    kernel applied it."""
    m = N - F
    faulty, init = shape(N, F, ties(m) if m % 2 else [1, 0] * (m // 2))
    seed = 0x5A + N
    net = benor.Network(N, F, init, faulty)
    net.start_live(seed=seed, k_max=k_max)
    snaps, posted, stopped = [], [], set()
    t0 = time.perf_counter()
    while net.poll() and time.perf_counter() - t0 < 30:
        if N == 1024 and len(snaps) == 8:
            net.stop_node(700)
            stopped.add(700)
        posted.append(set(stopped))
        snaps.append(net.get_states_at())
    net.wait()
    events = net.live_stop_events()
    final = net.get_states()
    mids = [e for _, e in snaps if e is not None]
    assert mids == sorted(mids)                        # snapshots follow the run
    checked = check_snapshots(N, F, faulty, init, seed, k_max, snaps, events, posted)
    print(f"N={N}: {checked} snapshots checked, deliveries {mids[:3]}..{mids[-3:]}")
    assert checked >= 1
    ref, _ = oracle.event_trials(N, F, faulty, seed=seed, trial_begin=0, trial_count=1, k_max=k_max,
                                 initial_values=init, crash_at=[None if v is None else v for v in events],
                                 want_states=True)
    want = ref.states
    if all(s["decided"] is True for s in want):
        want = [dict(s, killed=True) for s in want]
    for i in stopped:
        want[i] = dict(want[i], killed=True)
    assert final == want


def test_live_snapshot_after_the_run_is_final():
    """Once the run has ended, bo_get_states returns the final states and no
    delivery count; bo_consensus_poll reports it ended."""
    N, F = 10, 4
    faulty, init = shape(N, F, [1, 0, 1, 0, 1, 0])
    net = benor.Network(N, F, init, faulty)
    net.start_live(seed=11, k_max=16)
    t0 = time.perf_counter()
    while net.poll():
        assert time.perf_counter() - t0 < 10
    st, e = net.get_states_at()
    assert e is None
    ref, _ = oracle.event_trials(N, F, faulty, seed=11, trial_begin=0, trial_count=1, k_max=16,
                                 initial_values=init, want_states=True)
    assert st == ref.states


def test_reference_polling_pattern_reaches_finality():
    """__test__/tests/utils.ts:14-24 with benorconsensus.test.ts:153-160: poll
    getNodesState until reachedFinality -- the live run's snapshots, then its
    final states (F > 0: no auto-stop)."""
    N, F = 1024, 341
    faulty, init = shape(N, F, [1] * 400 + [0] * 283)
    benor.launchNetwork(N, F, init, faulty)
    benor.startConsensus(N, seed=5)
    t0 = time.perf_counter()
    states = benor.getNodesState(N)
    while time.perf_counter() - t0 < 2.0 and not benor.reachedFinality(states):
        time.sleep(0.001)
        states = benor.getNodesState(N)
    assert benor.reachedFinality(states)
    assert all(s["decided"] and s["x"] == 1 and s["k"] == 2 for s in states[F:])
    benor.waitConsensus(N)
