"""Throughput of the Ben-Or round loop on MI355X (BASELINE.json metric).

Workload (BASELINE configs[3], the metric's config): N = 1024 nodes, F = 341
crash-faulty (the first F node ids, as in src/start.ts:7-18), iid
Bernoulli(1/2) initial values from Philox, lockstep delivery (the reference's
semantics for its admissible inputs), k_max = 16.  One step = one launch of
`--trials` independent trials per GPU (default 10^8) + the RCCL all-reduce of
the outcome histogram.  Weak scaling: every rank runs its own global trial-id
range [(step * world + rank) * T, +T), so the merged histogram is independent
of the GPU count.

value  = live node-rounds simulated by all ranks / timed seconds (max over ranks)
         (a live node-round = one live node executing one R-phase and one
         P-phase: SURVEY §8d primary count)
roofline: per-receiver tally popcount words per live node-round (m = N - F
         live nodes: c1 in the R-phase; c1 in the P-phase when the binary vote
         count is odd -- no "?" proposal, c0 = m - c1 -- else c0 and c1: 2 or
         3 * ceil(m/32), 44 at the bench shape) / average kernel
         duration from HIP events on the launch stream, against the gfx950
         v_bcnt_u32_b32 issue peak (256 CU x 4 SIMD x 16 lanes x 2.4 GHz =
         39.3 T words/s).
cpu_baseline: the oracle's bit-plane restatement (oracle/benor_oracle.c,
         OpenMP over trials) on a bounded sample, rank 0 at N = 1 only.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, backend nccl = RCCL).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "ben-or-consensus-algorithm_amd")
sys.path.insert(0, PKG)

METRIC = "simulated node-rounds/sec at N=1024,F=341, 1–8 GPUs; % of INT/popcount roofline"
# v_bcnt_u32_b32 issues one wave64 instruction per 4 cycles per SIMD (16 lanes/clk;
# tools/valu_probe.hip, profiles/r01-v8_valu_probe.txt: 4.15-4.2 cyc at full occupancy,
# vs 2.4-2.5 for v_and_b32 / v_add_u32), so the popcount roofline of the chip is
# 256 CU x 4 SIMD x 16 lanes x 2.4 GHz.
SPEC_PEAK_POPC = 256 * 4 * 16 * 2.4e9


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--F", type=int, default=341)
    ap.add_argument("--trials", type=int, default=100_000_000, help="trials per GPU per step")
    ap.add_argument("--k-max", type=int, default=16)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x243F6A8885A308D3)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline sample budget (0 = skip)")
    ap.add_argument("--no-peak-probe", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true", help="skip the configs[1]/[2] side measurements")
    return ap.parse_args()


def node_rounds(hist, m, k_max):
    """Live node-rounds represented by a histogram: R rounds for a trial that
    halted after round R, k_max for an undecided one."""
    total_rounds = 0
    for R in range(1, k_max + 1):
        total_rounds += R * int(hist[R * 3] + hist[R * 3 + 1] + hist[R * 3 + 2])
    total_rounds += k_max * int(hist[0] + hist[1] + hist[2])
    return total_rounds * m, total_rounds


# BASELINE configs[1] and [2] (one GPU): measured after the timed region and
# reported beside the headline, not part of `value`.
OTHER_CONFIGS = [("C2 N=10,F=4", 10, 4, 1_000_000), ("C2 N=10,F=5 (F>N/2, no decision)", 10, 5, 1_000_000),
                 ("C3 N=256,F=85", 256, 85, 10_000_000)]


def other_configs(benor, torch, k_max, seed):
    import numpy as np

    stream = torch.cuda.current_stream()
    out = {}
    for name, N, F, T in OTHER_CONFIGS:
        plan = benor.TrialsPlan(N, F, [i < F for i in range(N)], seed=seed, k_max=k_max)
        h = torch.zeros(plan.hist_len, dtype=torch.int64, device="cuda")
        plan.launch(0, T, h.data_ptr(), stream.cuda_stream)          # warm-up launch
        torch.cuda.synchronize()
        h.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        plan.launch(T, T, h.data_ptr(), stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        hist = h.cpu().numpy().astype(np.uint64)
        nr, rounds = node_rounds(hist, plan.live_nodes, k_max)
        undecided = int(hist[0] + hist[1] + hist[2])
        out[name] = {"trials": T, "kernel_ms": ms, "node_rounds_per_s": nr / (ms * 1e-3),
                     "trials_per_s": T / (ms * 1e-3), "mean_rounds": rounds / T, "undecided_trials": undecided}
    return out


def cpu_baseline(N, F, k_max, seed, budget_s):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    faulty = [i < F for i in range(N)]
    m = N - F
    n = 100_000                     # calibration sample (~0.1 s on 16 threads)
    t0 = time.perf_counter()
    oracle.run_trials(N, F, faulty, seed=seed, trial_begin=0, trial_count=n, k_max=k_max, threads=threads)
    dt = time.perf_counter() - t0
    n2 = max(n, int(n * budget_s / max(dt, 1e-6)))
    t0 = time.perf_counter()
    r = oracle.run_trials(N, F, faulty, seed=seed, trial_begin=0, trial_count=n2, k_max=k_max, threads=threads)
    dt = time.perf_counter() - t0
    nr, _ = node_rounds(r.hist, m, k_max)
    return {"value": nr / dt, "unit": "node-rounds/s", "cores": threads, "kind": "port",
            "sample": f"{n2} trials of the bench workload (N={N}, F={F}, k_max={k_max}, same seed), "
                      f"{dt:.1f} s, oracle/benor_oracle.c bit-plane restatement, OpenMP over trials"}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import benor
    from benor.parallel import merge_histogram, weak_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; BENOR_DIST_BACKEND=gloo rehearses several ranks on one GPU
    backend = os.environ.get("BENOR_DIST_BACKEND", "nccl")
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    N, F, k_max, T = args.N, args.F, args.k_max, args.trials
    faulty = [i < F for i in range(N)]
    plan = benor.TrialsPlan(N, F, faulty, seed=args.seed, k_max=k_max)
    m = plan.live_nodes
    words_per_nr = plan.popc_words_per_node_round
    H = plan.hist_len
    stream = torch.cuda.current_stream()
    hist = torch.zeros(H, dtype=torch.int64, device="cuda")
    step_hist = torch.zeros(H, dtype=torch.int64, device="cuda")

    def step(s):
        step_hist.zero_()
        begin, n = weak_range(s, rank, world, T)
        plan.launch(begin, n, step_hist.data_ptr(), stream.cuda_stream)
        merge_histogram(step_hist)              # RCCL merge of the outcome histograms
        hist.add_(step_hist)

    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize()
    hist.zero_()
    # kernel-only timing with HIP events on the launch stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        s = args.warmup + i
        step_hist.zero_()
        begin, n = weak_range(s, rank, world, T)
        ev[i][0].record(stream)
        plan.launch(begin, n, step_hist.data_ptr(), stream.cuda_stream)
        ev[i][1].record(stream)
        merge_histogram(step_hist)
        hist.add_(step_hist)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    h = hist.cpu().numpy().astype(np.uint64)
    assert int(h.sum()) == T * world * args.steps, "histogram lost trials"
    live_nr, rounds = node_rounds(h, m, k_max)
    value = live_nr / elapsed
    # roofline of the dominant kernel (one launch = T trials on this rank)
    per_launch_nr = live_nr / (world * args.steps)
    avg_kernel_s = float(np.mean(kern_ms)) * 1e-3
    achieved = per_launch_nr * words_per_nr / avg_kernel_s
    peak_measured = None
    if not args.no_peak_probe:
        peak_measured = benor.popc_peak(10)
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):
        try:
            tj = json.load(open(tfile))
            if tj.get("N") == N and tj.get("F") == F and tj.get("trials") == T:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    out = {
        "metric": METRIC, "value": value, "unit": "node-rounds/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic (Philox initial values)",
        "config": {"workload": f"N={N},F={F} lockstep crash faults, {T} trials per GPU per step, k_max={k_max}",
                   "N": N, "F": F, "live_nodes": m, "trials_per_gpu_per_step": T, "k_max": k_max,
                   "parallelism": f"dp{world} (trial-id sharding, RCCL histogram all-reduce)"},
        "roofline": {"bound": "valu (v_bcnt_u32_b32 issue)", "achieved": achieved / 1e12, "peak": SPEC_PEAK_POPC / 1e12,
                     "unit": "Tpopc/s", "frac": achieved / SPEC_PEAK_POPC, "traffic": traffic,
                     "kernel_ms": float(np.mean(kern_ms)), "popc_words_per_node_round": words_per_nr,
                     "peak_probe": (peak_measured / 1e12) if peak_measured else None},
        "all_node_rounds_per_s": rounds * N / elapsed,
        "trials_per_s": T * world * args.steps / elapsed,
    }
    if world == 1 and not args.no_other_configs:
        out["other_configs"] = other_configs(benor, torch, k_max, args.seed)
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(N, F, k_max, args.seed, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
