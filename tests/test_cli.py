"""benor.cli: the start.ts scenario checks, the histogram
summary, and a small C5 sweep on the GPU compared with the analytic law."""
import csv
import os
import subprocess
import sys

import numpy as np
import pytest

import analytic
import oracle
from benor import Error
from benor.cli import main, summarize
from conftest import PKG


def test_summarize_matches_histogram():
    N, F, k = 10, 4, 16
    h = oracle.run_trials(N, F, [i < F for i in range(N)], seed=4, trial_count=50_000, k_max=k).hist
    row = summarize(h, N, F, k)
    assert row["trials"] == 50_000 and row["decided_frac"] == 1.0
    assert abs(row["E_R"] - analytic.expected_rounds(N, F)) < 0.02
    assert abs(row["P_R1"] - (1 - analytic.tie_prob(6))) < 0.01


def test_start_rejects_like_start_ts():
    with pytest.raises(Error, match="Too many faulty nodes"):          # start.ts:25-29
        main(["start", "--N", "4", "--faulty", "0,1,2", "--init", "1,1,1,1"])
    with pytest.raises(Error, match="Lengths don't match"):            # start.ts:22-23
        main(["start", "--N", "4", "--faulty", "0", "--init", "1,1,1"])


@pytest.mark.gpu
def test_start_scenario_runs(capsys):
    assert main(["start", "--seed", "7"]) == 0                         # N=10, nodes 0-3 faulty, all 1
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 10 and all('"decided": true' in line for line in out[4:])


@pytest.mark.gpu
def test_small_sweep_against_law(tmp_path):
    out = tmp_path / "sweep.csv"
    env = dict(os.environ, PYTHONPATH=PKG)
    subprocess.run([sys.executable, "-m", "benor.cli", "sweep", "--N", "64,128", "--steps", "4", "--trials",
                    str(8 * 200_000), "--out", str(out), "--k-max", "24"], check=True, env=env, cwd=PKG, timeout=120)
    rows = list(csv.DictReader(open(out)))
    assert len(rows) == 8
    for r in rows:
        N, F = int(r["N"]), int(r["F"])
        assert int(r["trials"]) == 200_000 and int(r["agreement_violations"]) == 0
        exp = 1 - analytic.tie_prob(N - F)
        sd = (exp * (1 - exp) / 200_000) ** 0.5
        assert abs(float(r["P_R1"]) - exp) < 6 * sd + 1e-9, r


@pytest.mark.gpu
def test_sweep_two_ranks_equals_one(tmp_path):
    """C5's multi-GPU path: each cell's trials split over ranks,
    one all-reduce of the [cells, H] histogram buffer.  Two ranks over gloo on
    one GPU must write the byte-identical CSV of one rank, since Philox is keyed
    by the global trial id."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    args = ["sweep", "--N", "64,1024,2112", "--steps", "3", "--trials", str(9 * 30_001), "--k-max", "12"]
    env = dict(os.environ, PYTHONPATH=PKG)
    one = tmp_path / "one.csv"
    subprocess.run([sys.executable, "-m", "benor.cli", *args, "--out", str(one)], check=True, env=env, cwd=PKG,
                   timeout=120)
    two = tmp_path / "two.csv"
    env2 = dict(env, BENOR_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                    "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "benor.cli", *args,
                    "--out", str(two)], check=True, env=env2, cwd=PKG, timeout=180)
    assert one.read_bytes() == two.read_bytes()
    rows = list(csv.DictReader(open(one)))
    assert len(rows) == 9 and all(int(r["trials"]) == 30_001 for r in rows)


@pytest.mark.gpu
def test_sweep_streams_equal_one_stream(tmp_path):
    """Cells spread over several streams (the default) write the byte-identical
    CSV of one stream: every plan owns its deferral buffers, so concurrent cells
    (including deferral chains at N=1024 / 2112 / 4096) are independent."""
    args = ["sweep", "--N", "64,1024,2112,4096", "--steps", "4", "--per-cell", str(3 * (1 << 20) + 17), "--k-max", "12"]
    env = dict(os.environ, PYTHONPATH=PKG)
    outs = []
    for streams in (1, 4, 3):
        out = tmp_path / f"s{streams}.csv"
        subprocess.run([sys.executable, "-m", "benor.cli", *args, "--streams", str(streams), "--out", str(out)],
                       check=True, env=env, cwd=PKG, timeout=120)
        outs.append(out.read_bytes())
    assert outs[0] == outs[1] == outs[2]
    assert len(outs[0].splitlines()) == 1 + 16
