"""Command-line driver.

    python -m benor.cli start [--N 10 --faulty 0,1,2,3 --init 1,1,...]   # src/start.ts
    python -m benor.cli trials --N 1024 --F 341 --trials 1000000          # one batch, JSON summary
    python -m benor.cli sweep --N 64,128,...,4096 --steps 32 --trials 2**30 --out sweep.csv
                                                                          # C5 phase diagram
    python -m benor.cli sweep --cells 4096:0,4096:1984 --per-cell 4793490  # two cells of it

`start` re-states src/start.ts:6-43: same default scenario (N = 10, nodes
0-3 faulty, every initial value 1), same checks ("Lengths don't match",
"Too many faulty nodes" when F > N/2), then launchNetwork + startConsensus,
and prints every node's state.

`sweep` runs the decision-round phase diagram: every N in the list crossed
with F = floor(phi * N), phi on a `--steps` grid in [0, 0.5); the total trial
budget is split evenly over cells, each cell's trials split across ranks
(torch.distributed, one process per GPU).  All cells are launched back to back
into one [cells, H] histogram buffer, merged with a single all-reduce.  Rows: N, F, m, trials, decided fraction, E[R], P(R = 1..4), P(v = 1),
undecided, agreement violations.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def _int(text: str) -> int:
    """A decimal integer, or a power written a**b (e.g. 2**30)."""
    base, sep, exp = text.strip().partition("**")
    return int(base) ** int(exp) if sep else int(base)


def _ints(s: str) -> list[int]:
    return [_int(part) for part in s.split(",") if part.strip()]


def summarize(hist: np.ndarray, N: int, F: int, k_max: int) -> dict:
    m = N - F
    trials = int(hist[:-1].sum())
    dec = np.array([int(hist[r * 3] + hist[r * 3 + 1] + hist[r * 3 + 2]) for r in range(1, k_max + 1)])
    decided = int(dec.sum())
    v1 = int(sum(hist[r * 3 + 1] for r in range(1, k_max + 1)))
    er = float((dec * np.arange(1, k_max + 1)).sum() / decided) if decided else float("nan")
    row = {"N": N, "F": F, "m": m, "trials": trials, "decided_frac": decided / trials if trials else 0.0,
           "E_R": er, "P_v1_given_decided": v1 / decided if decided else float("nan"),
           "undecided": int(hist[0] + hist[1] + hist[2]), "agreement_violations": int(hist[-1])}
    for r in range(1, 5):
        row[f"P_R{r}"] = (int(dec[r - 1]) / trials) if trials and r <= k_max else 0.0
    return row


def cmd_start(a) -> int:
    import benor

    N = a.N
    faulty_idx = set(_ints(a.faulty)) if a.faulty is not None else {0, 1, 2, 3}
    faulty = [i in faulty_idx for i in range(N)]
    init = [("?" if v == "?" else int(v)) for v in a.init.split(",")] if a.init else [1] * N
    if len(init) != len(faulty):                                   # start.ts:22-23
        raise benor.Error("Lengths don't match")
    if sum(faulty) > len(init) / 2:                                 # start.ts:25-29
        raise benor.Error("Too many faulty nodes")
    benor.launchNetwork(len(init), sum(faulty), init, faulty)       # start.ts:31-36
    benor.startConsensus(len(init), seed=a.seed, k_max=a.k_max)     # start.ts:40
    for i, s in enumerate(benor.getNodesState(len(init))):
        print(f"Node {i}: {json.dumps(s)}")
    return 0


def cmd_trials(a) -> int:
    import benor

    plan = benor.TrialsPlan(a.N, a.F, seed=a.seed, k_max=a.k_max)
    t0 = time.perf_counter()
    h = plan.run(a.begin, a.trials)
    dt = time.perf_counter() - t0
    row = summarize(h, a.N, a.F, a.k_max)
    row["seconds"] = dt
    print(json.dumps(row))
    return 0


def cmd_sweep(a) -> int:
    import torch

    import benor
    from benor.parallel import merge_histogram, strong_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist

        backend = os.environ.get("BENOR_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    if a.cells:
        # selected cells of a full sweep, re-run at that sweep's per-cell budget (--per-cell):
        # a cell's rows depend only on (N, F, seed, per-cell trials, k_max)
        cells = [tuple(_int(x) for x in c.split(":")) for c in a.cells.split(",")]
    else:
        cells = grid_cells(_ints(a.N), a.steps)
    per_cell = _int(str(a.per_cell)) if a.per_cell else max(1, _int(str(a.trials)) // len(cells))
    rows, elapsed = run_sweep(cells, per_cell, a.seed, a.k_max, a.streams, rank, world, a.progress)
    if rank == 0:
        out = open(a.out, "w") if a.out else sys.stdout
        out.write(rows_csv(rows))
        if a.out:
            out.close()
        total = per_cell * len(cells)
        print(json.dumps({"cells": len(cells), "trials": total, "seconds": elapsed, "gpus": world}), file=sys.stderr)
    return 0


def grid_cells(Ns: list[int], steps: int) -> list[tuple[int, int]]:
    """C5 cells: every N crossed with F = floor(phi N), phi on a `steps` grid in [0, 0.5)."""
    phis = [i * 0.5 / steps for i in range(steps)]
    return [(N, int(phi * N)) for N in Ns for phi in phis]


def rows_csv(rows: list[dict]) -> str:
    keys = list(rows[0].keys())
    return ",".join(keys) + "\n" + "".join(",".join(str(r[k]) for k in keys) + "\n" for r in rows)


def run_sweep(cells, per_cell, seed, k_max, streams_n=4, rank=0, world=1, progress=False):
    """The sweep's GPU work on the current device: (rows, seconds).  Under
    torch.distributed (world > 1) each cell's trials are split over the ranks
    and the histograms merged by one all-reduce."""
    import torch

    import benor
    from benor.parallel import merge_histogram, strong_range

    # The device context comes up before the clock starts (~0.08 s on a fresh
    # process): "seconds" times the sweep -- plans, launches, merge, read-back.
    torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stream = torch.cuda.current_stream()
    # Every cell's plan first, then all launches back to back into one [cells, H]
    # histogram buffer, then ONE all-reduce over ranks and one read-back.  Cells go
    # round-robin over --streams streams: each plan owns its buffers, so cells are
    # independent, and one cell's short passes (deferred-trial rounds, the last
    # groups of a launch) overlap the next cell's launches instead of idling CUs.
    plans = [benor.TrialsPlan(N, F, seed=seed ^ (N << 20) ^ F, k_max=k_max) for (N, F) in cells]
    H = plans[0].hist_len
    hists = torch.zeros((len(cells), H), dtype=torch.int64, device="cuda")
    streams = [stream] + [torch.cuda.Stream() for _ in range(max(1, streams_n) - 1)]
    for s in streams[1:]:
        s.wait_stream(stream)                      # the zeroed histograms
    b, n = strong_range(0, per_cell, rank, world)
    for ci, plan in enumerate(plans):
        plan.launch(b, n, hists[ci].data_ptr(), streams[ci % len(streams)].cuda_stream)
        if rank == 0 and progress:
            print(f"[{ci + 1}/{len(cells)}] N={cells[ci][0]} F={cells[ci][1]} queued", file=sys.stderr, flush=True)
    for s in streams[1:]:
        stream.wait_stream(s)
    merge_histogram(hists)
    allh = hists.cpu().numpy().astype(np.uint64)
    rows = [summarize(allh[ci], N, F, k_max) for ci, (N, F) in enumerate(cells)]
    elapsed = time.perf_counter() - t0
    for plan in plans:
        plan.check()                               # device-side capacity invariants of every cell
    return rows, elapsed


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="benor")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("start", help="src/start.ts scenario")
    s.add_argument("--N", type=int, default=10)
    s.add_argument("--faulty", default=None, help="comma-separated faulty node ids (default 0,1,2,3)")
    s.add_argument("--init", default=None, help="comma-separated initial values 0/1/? (default all 1)")
    s.add_argument("--seed", type=int, default=None)
    s.add_argument("--k-max", type=int, default=64)
    t = sub.add_parser("trials", help="one batch of independent trials")
    t.add_argument("--N", type=int, default=1024)
    t.add_argument("--F", type=int, default=341)
    t.add_argument("--trials", type=int, default=1_000_000)
    t.add_argument("--begin", type=int, default=0)
    t.add_argument("--seed", type=int, default=0x243F6A8885A308D3)
    t.add_argument("--k-max", type=int, default=16)
    w = sub.add_parser("sweep", help="C5 decision-round phase diagram")
    w.add_argument("--N", default="64,128,256,512,1024,2048,4096")
    w.add_argument("--steps", type=int, default=32)
    w.add_argument("--trials", default="2**30")
    w.add_argument("--seed", type=int, default=0x243F6A8885A308D3)
    w.add_argument("--k-max", type=int, default=32)
    w.add_argument("--cells", default=None, help="N:F,N:F,... instead of the N x phi grid")
    w.add_argument("--per-cell", default=None, help="trials per cell (default: --trials / cells)")
    w.add_argument("--streams", type=int, default=4, help="HIP streams the cells are spread over")
    w.add_argument("--out", default=None)
    w.add_argument("--progress", action="store_true")
    a = ap.parse_args(argv)
    return {"start": cmd_start, "trials": cmd_trials, "sweep": cmd_sweep}[a.cmd](a)


if __name__ == "__main__":
    sys.exit(main())
