"""Matrix-core kernel check on one GPU: histograms against the oracle (small
trial counts) and against the popcount W kernel (BENOR_NO_MFMA=1, large
counts), then launch timing of both on the BASELINE shapes.

Run from the repo root: python tools/mfma_check.py > gpurun_out/mfma_check.jsonl
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ben-or-consensus-algorithm_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import benor  # noqa: E402
import oracle  # noqa: E402


def plan(N, F, mfma, **kw):
    if mfma:
        os.environ.pop("BENOR_NO_MFMA", None)
    else:
        os.environ["BENOR_NO_MFMA"] = "1"
    p = benor.TrialsPlan(N, F, **kw)
    os.environ.pop("BENOR_NO_MFMA", None)
    return p


def emit(**d):
    print(json.dumps(d), flush=True)


def shapes():
    out = []
    for W in range(2, 17):
        for off in (1, 33, 63):
            m = 64 * (W - 1) + off
            if m > 1024 or m % 2 == 0:
                continue
            for F in ((m - 1) // 2, (m - 1) // 3):
                out.append((m + F, F))
    return out


def main():
    bad = 0
    # oracle parity, random init
    for i, (N, F) in enumerate(shapes()):
        seed = 1000 + i
        T = 1000 + 37 * (i % 5)
        got = plan(N, F, True, seed=seed, k_max=8).run(123 + i, T)
        ref = oracle.run_trials(N, F, [j < F for j in range(N)], seed=seed, trial_begin=123 + i,
                                trial_count=T, k_max=8)
        ok = bool(np.array_equal(got, ref.hist))
        bad += not ok
        emit(check="oracle", N=N, F=F, m=N - F, trials=T, ok=ok)
    # fixed init with an even number of "?" (M = m - init_q odd)
    for N, F, q in ((300, 99, 2), (1024, 341, 10), (129, 40, 4)):
        rng = np.random.default_rng(N)
        vals = [int(v) for v in rng.integers(0, 2, N)]
        live = list(range(F, N))
        for j in rng.choice(live, q, replace=False):
            vals[j] = "?"
        got = plan(N, F, True, seed=7, k_max=8, initial_values=vals).run(0, 333)
        ref = oracle.run_trials(N, F, [j < F for j in range(N)], seed=7, trial_begin=0, trial_count=333, k_max=8,
                                initial_values=vals)
        ok = bool(np.array_equal(got, ref.hist))
        bad += not ok
        emit(check="oracle_fixed", N=N, F=F, q=q, ok=ok)
    # against the popcount kernel, 10^6 trials
    for N, F in ((1024, 341), (256, 85), (1000, 300), (97, 32)):
        a = plan(N, F, True, seed=99, k_max=16).run(5, 1_000_003)
        b = plan(N, F, False, seed=99, k_max=16).run(5, 1_000_003)
        ok = bool(np.array_equal(a, b))
        bad += not ok
        emit(check="vs_w_kernel", N=N, F=F, trials=1_000_003, ok=ok, hist=[int(x) for x in a[:8]])
    # timing
    for N, F, T in ((1024, 341, 100_000_000), (256, 85, 200_000_000)):
        for mf in (True, False):
            p = plan(N, F, mf, seed=1, k_max=16)
            p.run(0, T // 10)
            t0 = time.perf_counter()
            h = p.run(0, T)
            dt = time.perf_counter() - t0
            emit(check="timing", N=N, F=F, mfma=mf, trials=T, s=dt, node_rounds_per_s=T * (N - F) / dt,
                 hist=[int(x) for x in h[:8]])
    emit(check="done", bad=bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
