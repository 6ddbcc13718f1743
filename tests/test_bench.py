"""bench.py contract: one JSON line with the BASELINE metric, roofline and
(at N=1) cpu_baseline; the multi-rank path (trial sharding + histogram
all-reduce + max-over-ranks timing) rehearsed with two ranks on one GPU over
gloo (the driver's 8-GPU runs use the same code with backend nccl = RCCL)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_helpers():
    sys.path.insert(0, ROOT)
    import numpy as np

    import bench

    k = 4
    h = np.zeros((k + 1) * 3 + 1, dtype=np.uint64)
    h[1 * 3 + 0] = 5          # 5 trials halted after round 1
    h[3 * 3 + 1] = 2          # 2 after round 3
    h[0] = 1                  # 1 undecided after k rounds
    live_nr, rounds = bench.node_rounds(h, m=7, k_max=k)
    assert rounds == 5 * 1 + 2 * 3 + 1 * k
    assert live_nr == rounds * 7


@pytest.mark.gpu
def test_bench_single_gpu_line():
    env = dict(os.environ)
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--trials", "4000000",
                        "--cpu-seconds", "1", "--no-peak-probe"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["unit"] == "node-rounds/s"
    assert 0 < d["roofline"]["frac"] < 1.0
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["kind"] == "port"
    # BASELINE configs[1] and [2] beside the headline
    oc = d["other_configs"]
    assert oc["C2 N=10,F=4"]["undecided_trials"] == 0 and oc["C2 N=10,F=4"]["mean_rounds"] > 1.3
    assert oc["C2 N=10,F=5 (F>N/2, no decision)"]["undecided_trials"] == 1_000_000
    assert oc["C3 N=256,F=85"]["mean_rounds"] == 1.0 and oc["C3 N=256,F=85"]["node_rounds_per_s"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [2, 4])
def test_bench_ranks_gloo_one_gpu(ranks):
    env = dict(os.environ, BENOR_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", str(ranks),
           "--steps", "2", "--warmup", "1", "--trials", "1000000", "--no-peak-probe"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == ranks and d["scaling"] == "weak"
    # every rank ran its own 10^6 trials per step; rank 0's merged histogram saw them all
    assert d["trials_per_s"] * d["ms_per_step"] * 1e-3 == pytest.approx(ranks * 1_000_000, rel=1e-6)
    assert "cpu_baseline" not in d
    assert "other_configs" not in d
