"""Summarise a BENOR_TIMELINE file (the packed matrix-core kernel's per-wave
phase stamps, benor_mfma_small.h) -- the last launch in the file.

    python tools/timeline_report.py <file> [--run N F TRIALS]

--run first launches N, F, TRIALS (random init, k_max 16) twice through the C
ABI with BENOR_TIMELINE=<file> (GPU; the first launch warms up).

Stamps are the 100 MHz wall clock (10 ns ticks).  Per wave: [0] start, [1]
fresh round-1 batches exhausted, [2] round lists drained, [3] lane path done,
[4] histogram flushed; counts: fresh, r2 full, r3 full, r2 partial, r3
partial, lane-path passes.
"""
import os
import statistics
import sys


def last_launch(path):
    head, rows = None, []
    for line in open(path):
        if line.startswith("#"):
            head, rows = line.strip(), []
        elif line.strip():
            rows.append([int(x) for x in line.split(",")])
    return head, rows


def q(xs, f):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(f * len(xs)))]


def report(path):
    head, rows = last_launch(path)
    rows = [r for r in rows if r[1]]                  # waves that ran
    t0 = min(r[1] for r in rows)
    us = lambda t: (t - t0) / 100.0
    print(head, f"({len(rows)} waves ran)")
    cols = [("start", 1), ("fresh done", 2), ("lists drained", 3), ("lane path done", 4), ("flushed", 5)]
    print("| phase end (us after the first wave's start) | min | median | p90 | max |")
    print("|---|---|---|---|---|")
    for name, i in cols:
        xs = [us(r[i]) for r in rows]
        print(f"| {name} | {min(xs):.2f} | {statistics.median(xs):.2f} | {q(xs, 0.9):.2f} | {max(xs):.2f} |")
    print("| phase length (us) | min | median | p90 | max |")
    print("|---|---|---|---|---|")
    for (a, i), (b, j) in zip(cols, cols[1:]):
        xs = [(r[j] - r[i]) / 100.0 for r in rows]
        print(f"| {a} -> {b} | {min(xs):.2f} | {statistics.median(xs):.2f} | {q(xs, 0.9):.2f} | {max(xs):.2f} |")
    names = ["fresh", "r2 full", "r3 full", "r2 partial", "r3 partial", "lane passes"]
    print("| batches per wave | min | mean | max |")
    print("|---|---|---|---|")
    for k, nm in enumerate(names):
        xs = [r[6 + k] for r in rows]
        print(f"| {nm} | {min(xs)} | {sum(xs) / len(xs):.2f} | {max(xs)} |")
    last = max(rows, key=lambda r: r[5])
    print("slowest wave:", {n: last[6 + k] for k, n in enumerate(names)},
          "phases (us):", [round(us(last[i]), 2) for _, i in cols])


def run(path, N, F, trials):
    os.environ["BENOR_TIMELINE"] = path
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ben-or-consensus-algorithm_amd"))
    import benor
    faulty = [i < F for i in range(N)]
    for _ in range(2):
        plan = benor.TrialsPlan(N, F, faulty, seed=7, k_max=16)
        plan.run(0, trials)


if __name__ == "__main__":
    path = sys.argv[1]
    if len(sys.argv) > 2 and sys.argv[2] == "--run":
        if os.path.exists(path):
            os.remove(path)
        run(path, int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
    report(path)
