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


def test_bench_self_launch_dry_run():
    """`bench.py --gpus 2` without a launcher starts two ranks itself; every
    rank sees WORLD_SIZE=2 and the strong-scaling shards partition each step."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1",
                        "--trials", "1001"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = sorted((json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")), key=lambda d: d["rank"])
    assert [d["rank"] for d in lines] == [0, 1] and all(d["world"] == 2 for d in lines)
    for i in range(2):
        (b0, n0), (b1, n1) = lines[0]["shards"][i], lines[1]["shards"][i]
        assert b0 == (1 + i) * 1001 and b0 + n0 == b1 and n0 + n1 == 1001


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--dry-run"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


@pytest.mark.parametrize("knob", ["BENOR_NO_MFMA", "BENOR_BLOCKS_PER_CU", "BENOR_TIMELINE"])
def test_bench_refuses_libbenor_knobs(knob):
    """A knob that forces a kernel, a grid or a test path makes bench.py exit
    before any GPU work: a figure is only reported for the
    planner's own kernels."""
    env = dict(os.environ, **{knob: "1"})
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "0"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and knob in r.stderr and "refusing" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def _run_bench(args, env_extra=None, launcher=None, timeout=300):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **(env_extra or {}))
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable] + (launcher or []) + ["bench.py"] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return _json_line(r.stdout)


@pytest.mark.gpu
def test_bench_single_gpu_line():
    d = _run_bench(["--steps", "2", "--warmup", "1", "--trials", "4000000", "--cpu-seconds", "1", "--no-peak-probe"])
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["unit"] == "node-rounds/s" and d["scaling"] == "strong"
    assert 0 < d["roofline"]["frac"] < 1.0
    assert d["dist"]["world"] == 1 and d["dist"]["backend"] is None and d["agreement_violations"] == 0
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["kind"] == "port"
    assert d["cpu_baseline"]["single_core"]["cores"] == 1 and d["cpu_baseline"]["single_core"]["value"] > 0
    # BASELINE configs[1] and [2] beside the headline, each with its roofline
    oc = d["other_configs"]
    assert oc["C2 N=10,F=4"]["undecided_trials"] == 0 and oc["C2 N=10,F=4"]["mean_rounds"] > 1.3
    assert oc["C2 N=10,F=5 (F>N/2, no decision)"]["undecided_trials"] == 1_000_000
    assert oc["C3 N=256,F=85"]["mean_rounds"] == 1.0 and oc["C3 N=256,F=85"]["node_rounds_per_s"] > 0
    # configs[4] cells at N=4096 (cooperative big-network kernel): m odd halts in round 1;
    # m even is a deferral chain per launch, timed as a whole
    c5a, c5b = oc["C5 cell N=4096,F=1365"], oc["C5 cell N=4096,F=0"]
    assert c5a["mean_rounds"] == 1.0 and "kernels_per_launch" not in c5a
    assert c5b["kernels_per_launch"] and c5b["undecided_trials"] == 0 and 1.0 < c5b["mean_rounds"] < 1.05
    c1 = oc.pop("C1 N=5,F=1 network API")                 # configs[0]: one network, reference calls
    for leg in ("default", "sync"):
        assert c1[leg]["reference_assertions_hold"] and 0 < c1[leg]["median_ms"] < 50
    net = oc.pop("C4 N=1024,F=341 network API, mid-run /stop")   # one network through the drop-in API
    assert net["stop inside round 1"]["stopped_nodes"] == 1 and net["stop inside round 1"]["seconds"] > 0
    assert net["no stop, sync start (lockstep kernel)"]["stopped_nodes"] == 0
    live = net["default (live) start, /stop sent after it"]
    assert live["stopped_nodes"] == 1 and live["stop_landed_at_delivery"] is not None
    assert live["start_returned_after_s"] < live["seconds"]
    sweep = oc.pop("C5 sweep (2^30 trials, 224 cells)")          # configs[4] end to end, CSV checked
    assert sweep["cells"] == 224 and sweep["trials"] > 2 ** 29 and sweep["csv_equals_results_r02_sweep_c5"] is True
    for k, v in oc.items():
        assert 0 < v["roofline"]["frac"] < 1.0 and v["roofline"]["bound"], k
    # N=256/F=85 and the headline run on the matrix cores (m odd, m > 2F): 2m terms per node-round
    assert oc["C3 N=256,F=85"]["roofline"]["terms_per_node_round"] == 2 * 171
    assert d["roofline"]["kernel"].startswith("matrix core") and d["roofline"]["terms_per_node_round"] == 2 * 683
    assert d["roofline"]["unit"] == "TFLOP/s" and 0.9 < d["roofline"]["padding_efficiency"] <= 1.0


@pytest.mark.gpu
def test_bench_nccl_world_one_under_launcher():
    """The RCCL branch: torch.distributed.run with one rank, backend nccl."""
    d = _run_bench(["--gpus", "1", "--steps", "2", "--warmup", "1", "--trials", "1000000", "--no-peak-probe",
                    "--no-other-configs", "--cpu-seconds", "0"],
                   launcher=["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                             "--master-addr", "127.0.0.1", "--master-port", str(_free_port())])
    assert d["n_gpus"] == 1 and d["dist"] == {**d["dist"], "world": 1, "backend": "nccl", "ranks_merged_per_step": 1}


@pytest.mark.gpu
@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_bench_self_launched_ranks_match_one_rank(scaling):
    """`bench.py --gpus 2` (no launcher; two ranks on one GPU over gloo) reports
    n_gpus 2 and merges a histogram bit-identical to one rank running the same
    trial ids."""
    common = ["--steps", "2", "--warmup", "1", "--no-peak-probe", "--no-other-configs", "--cpu-seconds", "0"]
    T = 1_000_000
    one = _run_bench(["--gpus", "1", "--scaling", scaling, "--trials", str(T if scaling == "strong" else 2 * T)]
                     + common)
    two = _run_bench(["--gpus", "2", "--scaling", scaling, "--trials", str(T)] + common,
                     env_extra={"BENOR_DIST_BACKEND": "gloo"})
    assert two["n_gpus"] == 2 and two["dist"]["world"] == 2 and two["dist"]["ranks_merged_per_step"] == 2
    assert two["dist"]["backend"] == "gloo" and two["scaling"] == scaling
    assert two["dist"]["hist_sha256"] == one["dist"]["hist_sha256"]
    assert two["trials_per_s"] * two["ms_per_step"] * 1e-3 == pytest.approx(2 * T if scaling == "weak" else T,
                                                                             rel=1e-6)


@pytest.mark.gpu
def test_bench_four_ranks_gloo_one_gpu():
    d = _run_bench(["--gpus", "4", "--steps", "2", "--warmup", "1", "--trials", "1000000", "--no-peak-probe"],
                   env_extra={"BENOR_DIST_BACKEND": "gloo"},
                   launcher=["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
                             "--master-addr", "127.0.0.1", "--master-port", str(_free_port())])
    assert d["n_gpus"] == 4 and d["dist"]["ranks_merged_per_step"] == 4
    assert "cpu_baseline" not in d and "other_configs" not in d
