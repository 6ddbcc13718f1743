"""BASELINE configs[4] (C5 phase diagram) pinned by tests.

CPU: the committed sweep `results/r02_sweep_c5.csv` (2^30 trials over 224 cells,
N in {64..4096} x F = floor(phi N), phi = i/64) obeys the exact law of the
reference round loop (oracle/analytic.py): every cell decides
(m = N - F > N/2 > F), with zero agreement violations; P(R = 1) = 1 - q(m) and
P(R = 2) = q(m)(1 - q(m)) with q(m) = C(m, m/2) / 2^m for even m (0 for odd m:
R = 1 always); the decided value is a fair coin.  Each statistic is checked per
cell at 6 sigma and jointly by a chi-square over the cells.

GPU: two N = 4096 cells (the big-network matrix-core kernel, KIND 1) and one
N = 64 cell re-run through `python -m benor.cli sweep --cells` at the sweep's
per-cell budget reproduce the committed rows byte for byte.
"""
import csv
import math
import os
import subprocess
import sys

import pytest

import analytic
from conftest import PKG, ROOT

CSV = os.path.join(ROOT, "results", "r02_sweep_c5.csv")
PER_CELL = 2 ** 30 // 224


def rows():
    with open(CSV) as f:
        return list(csv.DictReader(f))


def test_c5_grid_and_budget():
    rs = rows()
    assert len(rs) == 224
    cells = [(int(r["N"]), int(r["F"])) for r in rs]
    grid = [(N, int(i * 0.5 / 32 * N)) for N in (64, 128, 256, 512, 1024, 2048, 4096) for i in range(32)]
    assert cells == grid
    for r in rs:
        assert int(r["trials"]) == PER_CELL
        assert int(r["m"]) == int(r["N"]) - int(r["F"])


def test_c5_every_cell_decides_and_agrees():
    for r in rs_decidable():
        assert float(r["decided_frac"]) == 1.0 and int(r["undecided"]) == 0, r
        assert int(r["agreement_violations"]) == 0, r


def rs_decidable():
    rs = rows()
    assert all(int(r["m"]) > int(r["F"]) for r in rs)     # F < N/2 on the grid: every cell can decide
    return rs


def z(p_hat, p, n):
    if p in (0.0, 1.0):
        return 0.0 if p_hat == p else math.inf
    return (p_hat - p) / math.sqrt(p * (1 - p) / n)


def test_c5_rounds_law_per_cell_and_joint():
    """P(R=1) = 1 - q, P(R=2) = q (1 - q), per cell at 6 sigma and
    jointly (sum of z^2 over the even-m cells against chi-square with that many
    degrees of freedom, at 6 standard deviations)."""
    chi, df = 0.0, 0
    for r in rs_decidable():
        m, n = int(r["m"]), int(r["trials"])
        q = analytic.tie_prob(m)
        z1 = z(float(r["P_R1"]), 1 - q, n)
        z2 = z(float(r["P_R2"]), q * (1 - q), n)
        assert abs(z1) < 6 and abs(z2) < 6, (r, z1, z2)
        if m % 2 == 0:
            chi += z1 * z1
            df += 1
        else:
            assert float(r["P_R1"]) == 1.0 and float(r["E_R"]) == 1.0, r
        er = (1.0 / (1 - q)) if q < 1 else math.inf                    # E[R] of the geometric law
        sd_er = math.sqrt(q) / (1 - q) / math.sqrt(n)
        assert abs(float(r["E_R"]) - er) < 6 * sd_er + 1e-12, r
    assert df == 16 + 6 * 32                 # N = 64: F = i, 16 even m; N >= 128: F = (N/64) i, m always even
    assert chi < df + 6 * math.sqrt(2 * df), (chi, df)


def test_c5_decided_value_is_fair():
    chi = 0.0
    for r in rs_decidable():
        n = int(r["trials"])
        zz = z(float(r["P_v1_given_decided"]), 0.5, n)
        assert abs(zz) < 6, r
        chi += zz * zz
    assert chi < 224 + 6 * math.sqrt(2 * 224)


@pytest.mark.gpu
def test_c5_cells_rerun_byte_identical(tmp_path):
    """Three committed cells re-run on the GPU at the sweep's per-cell budget:
    N = 4096, F = 0 and F = 1984 (big-network matrix-core kernel + deferral),
    N = 64, F = 20 (lane kernel).  The cell's histogram depends only on
    (N, F, seed, per-cell trials, k_max), so the rows must be byte-identical."""
    want = {}
    with open(CSV) as f:
        header = f.readline()
        for line in f:
            N, F = line.split(",")[:2]
            want[(int(N), int(F))] = line
    cells = [(4096, 0), (4096, 1984), (64, 20)]
    out = tmp_path / "cells.csv"
    env = dict(os.environ, PYTHONPATH=PKG)
    subprocess.run([sys.executable, "-m", "benor.cli", "sweep", "--cells", ",".join(f"{N}:{F}" for N, F in cells),
                    "--per-cell", str(PER_CELL), "--out", str(out)], check=True, env=env, cwd=PKG, timeout=120)
    got = open(out).read().splitlines(keepends=True)
    assert got[0] == header
    for (N, F), line in zip(cells, got[1:]):
        assert line == want[(N, F)], (N, F, line, want[(N, F)])
