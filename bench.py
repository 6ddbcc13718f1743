"""Throughput of the Ben-Or round loop on MI355X (BASELINE.json metric).

Workload (BASELINE configs[3], the metric's config): N = 1024 nodes, F = 341
crash-faulty (the first F node ids, as in src/start.ts:7-18), iid
Bernoulli(1/2) initial values from Philox, lockstep delivery (the reference's
semantics for its admissible inputs), k_max = 16.  One step = one launch per
GPU + the RCCL all-reduce of the outcome histogram.

  --scaling strong (default; configs[3] as written): every step runs 10^8
         trials in total, split into `world` contiguous shards of global
         trial ids [step * T, +T) (benor.parallel.strong_range);
  --scaling weak: every rank runs its own T trials per step, global ids
         [(step * world + rank) * T, +T).
Philox counters are keyed by the global trial id, so the merged histogram
depends only on the set of trial ids, never on the GPU count (`hist_sha256`).

value  = live node-rounds simulated by all ranks / timed seconds (max over ranks)
         (a live node-round = one live node executing one R-phase and one
         P-phase: SURVEY §8d primary count)
roofline: of the kernel the plan picked, from the average kernel duration
         (HIP events on the launch stream).  The bench shape runs the
         matrix-core kernel: algorithmic e2m1 FLOP/s -- every
         live receiver sums the m live votes in each phase, 4m FLOP per live
         node-round -- against the dense FP4 peak (~10 PFLOP/s).  A --N/--F
         shape the matrix cores do not take runs a popcount kernel: tally
         popcount words per live node-round (2 or 3 * ceil(m/32); DESIGN.md
         §4) against the v_bcnt_u32_b32 issue peak (256 CU x 4 SIMD x 16
         lanes x 2.4 GHz = 39.3 T words/s).
Environment: every BENOR_* variable set is recorded in the line ("env"); a
         libbenor knob (benor.KNOBS: forced kernels, grids, test paths) makes
         bench.py refuse to run -- a figure is only reported for the kernels
         the planner picks by itself.
cpu_baseline: the oracle's bit-plane restatement (oracle/benor_oracle.c,
         OpenMP over trials) on a bounded sample, rank 0 at N = 1 only, on
         every host thread and on one core.

Launch: python bench.py [--gpus N --steps K --warmup W].  For N > 1 the
driver starts it under torch.distributed.run (one process per GPU, backend
nccl = RCCL); started without a launcher, bench.py starts the N ranks itself
(before touching the GPU) and exits with their status.  A WORLD_SIZE that
differs from --gpus is an error, never a silent single-GPU run.
"""
import argparse
import hashlib
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "ben-or-consensus-algorithm_amd")
sys.path.insert(0, PKG)

METRIC = "simulated node-rounds/sec at N=1024,F=341, 1–8 GPUs; % of INT/popcount roofline"
# v_bcnt_u32_b32 issues one wave64 instruction per 4 cycles per SIMD (16 lanes/clk;
# tools/valu_probe.hip, profiles/r01-v8_valu_probe.txt: 4.15-4.2 cyc at full occupancy,
# vs 2.4-2.5 for v_and_b32 / v_add_u32), so the popcount roofline of the chip is
# 256 CU x 4 SIMD x 16 lanes x 2.4 GHz.  The same figure is the chip's VALU
# lane-op issue peak for 4-cycle VALU ops (v_cmp, SGPR-operand ops, Philox's
# v_mad_u64_u32 / v_bitop3_b32), used for the small-network kernel.
SPEC_PEAK_POPC = 256 * 4 * 16 * 2.4e9
# Matrix-core kernel (BO_KERNEL_MFMA): v_mfma_scale_f32_32x32x64_f8f6f4 on e2m1
# operands; dense FP4 peak ~10 PFLOP/s (MI355X_MICROARCH.md, Matrix cores),
# i.e. 5e15 receiver-sender multiply-adds per second.
SPEC_PEAK_MFMA_FLOPS = 10e15


def mfma_roofline(m, node_rounds_per_launch, kernel_s):
    """Roofline of the matrix-core kernel.  Algorithmic work: every live
    receiver sums the votes of the m live senders in the R- and the P-phase,
    2m multiply-adds (4m FLOP) per live node-round.  Executed work adds the
    padding of 32-row receiver tiles and 64-sender chunks: per 32-trial tile
    ceil(m/32) * (ceil(m/64) + ceil(ceil(m/32)/2)) instructions of 65536
    multiply-adds (benor_mfma.h)."""
    mt, w = (m + 31) // 32, (m + 63) // 64
    executed_per_trial = mt * (w + (mt + 1) // 2) * 65536 / 32
    flops = node_rounds_per_launch * 4 * m / kernel_s
    return {"bound": "mfma (v_mfma_scale_f32_32x32x64_f8f6f4, e2m1 0/1 operands)", "kernel": "matrix core",
            "achieved": flops / 1e12, "peak": SPEC_PEAK_MFMA_FLOPS / 1e12, "unit": "TFLOP/s",
            "frac": flops / SPEC_PEAK_MFMA_FLOPS, "terms_per_node_round": 2 * m,
            "padding_efficiency": 2 * m * m / executed_per_trial}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong: --trials in total per step, split over the ranks (configs[3]); "
                         "weak: --trials per rank per step")
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--F", type=int, default=341)
    ap.add_argument("--trials", type=int, default=100_000_000)
    ap.add_argument("--k-max", type=int, default=16)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x243F6A8885A308D3)
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="CPU-baseline sample budget on all host threads (0 = skip); the 1-core leg gets 2/3 of it")
    ap.add_argument("--no-peak-probe", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true", help="skip the configs[1]/[2] side measurements")
    ap.add_argument("--dry-run", action="store_true",
                    help="print this rank's place in the launch (world, rank, trial shards) and exit before any GPU work")
    return ap.parse_args(argv)


def node_rounds(hist, m, k_max):
    """Live node-rounds represented by a histogram: R rounds for a trial that
    halted after round R, k_max for an undecided one."""
    total_rounds = 0
    for R in range(1, k_max + 1):
        total_rounds += R * int(hist[R * 3] + hist[R * 3 + 1] + hist[R * 3 + 2])
    total_rounds += k_max * int(hist[0] + hist[1] + hist[2])
    return total_rounds * m, total_rounds


def hist_digest(hist):
    """Digest of a merged outcome histogram (uint64 little-endian bins)."""
    import numpy as np

    return hashlib.sha256(np.asarray(hist, dtype="<u8").tobytes()).hexdigest()[:16]


def rank_range(scaling, step, rank, world, trials):
    from benor.parallel import strong_range, weak_range

    if scaling == "strong":
        return strong_range(step * trials, trials, rank, world)
    return weak_range(step, rank, world, trials)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n, argv):
    """Start n ranks of this script under torch.distributed.run (one process
    per GPU) and return their exit status.  Called before anything here
    touches the GPU; the children are separate processes (no exec)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd, env=env).returncode


# BASELINE configs[1] and [2] (one GPU): measured after the timed region and
# reported beside the headline, not part of `value`.
OTHER_CONFIGS = [("C2 N=10,F=4", 10, 4, 1_000_000), ("C2 N=10,F=5 (F>N/2, no decision)", 10, 5, 1_000_000),
                 ("C3 N=256,F=85", 256, 85, 10_000_000),
                 # configs[4] (C5) cells at N = 4096 on the big-network matrix-core kernel
                 # (workgroup-cooperative form): KIND 0 (m odd, one launch per plan launch)
                 # and KIND 1 (m even: round 1, two continuation passes, the popcount
                 # remainder -- the line times all of them)
                 ("C5 cell N=4096,F=1365", 4096, 1365, 400_000), ("C5 cell N=4096,F=0", 4096, 0, 100_000)]
OTHER_REPS = 10          # back-to-back launches per config, each of its T trials
SS_REPS = 5              # back-to-back steady-state launches (20 T trials each)


def other_configs(benor, torch, k_max, seed):
    """One launch per config, HIP-event kernel time, and the roofline of the
    kernel that runs it:
      * m > 32 (W kernel): popcount words per live node-round
        (bo_plan_popc_words_per_node_round) against the v_bcnt issue peak;
      * m <= 64 (lane kernel, one trial per lane): VALU issue.
        Its algorithmic lane-ops per live node-round are the tally popcounts
        (2 or 3 one-word counts), the proposal compare, the decision compare
        and the all-decided check (3), plus one Philox4x32-10 word per coin
        flip (41 lane-ops per 4-word block).  Coins are flipped
        by every live node in every tie round; a deciding trial that halted
        after round R had R - 1 of them (an R-phase tie is the only way not to
        decide when N > 2F).  Undecided trials are counted with
        none, so the figure is a lower bound when they exist."""
    import numpy as np

    stream = torch.cuda.current_stream()
    out = {}
    for name, N, F, T in OTHER_CONFIGS:
        plan = benor.TrialsPlan(N, F, [i < F for i in range(N)], seed=seed, k_max=k_max)
        h = torch.zeros(plan.hist_len, dtype=torch.int64, device="cuda")
        plan.launch(0, T, h.data_ptr(), stream.cuda_stream)          # warm-up launch
        torch.cuda.synchronize()
        h.zero_()
        # A launch of 10^6 trials lasts tens of microseconds: timed alone, the
        # host's enqueue latency after the start event would count as kernel
        # time.  So OTHER_REPS launches of T distinct trials each go back to back
        # between the events, and kernel_ms is their average.
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for r in range(OTHER_REPS):
            plan.launch((1 + r) * T, T, h.data_ptr(), stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / OTHER_REPS
        hist = h.cpu().numpy().astype(np.uint64)
        m = plan.live_nodes
        nr, rounds = node_rounds(hist, m, k_max)             # per launch: the histogram holds OTHER_REPS launches
        nr, rounds = nr / OTHER_REPS, rounds / OTHER_REPS
        undecided = int(hist[0] + hist[1] + hist[2]) // OTHER_REPS
        words = plan.popc_words_per_node_round
        if plan.kernel == benor.BO_KERNEL_MFMA:
            roof = mfma_roofline(m, nr, ms * 1e-3)
            # the same rate against the INT/popcount roofline the metric names
            # (the popcount kernel's algorithmic words per node-round; >1: past it)
            roof["popcount_equiv"] = {"words_per_node_round": words,
                                      "frac_of_popc_peak": nr * words / (ms * 1e-3) / SPEC_PEAK_POPC}
        elif m > 64:
            roof = {"bound": "valu (v_bcnt_u32_b32 issue)", "kernel": "lockstep W kernel",
                    "unit": "Tpopc/s", "popc_words_per_node_round": words,
                    "achieved": nr * words / (ms * 1e-3) / 1e12}
        else:
            decided = T - undecided
            tie_rounds = (rounds - k_max * undecided) - decided
            ops = nr * (words + 3) + tie_rounds * m * 41 / 4
            roof = {"bound": "valu issue (tallies, compares, Philox coins)", "kernel": benor.KERNEL_NAMES[plan.kernel],
                    "unit": "T lane-ops/s", "lane_ops_per_node_round": ops / max(nr, 1),
                    "achieved": ops / (ms * 1e-3) / 1e12}
        if plan.kernel != benor.BO_KERNEL_MFMA:
            roof["peak"] = SPEC_PEAK_POPC / 1e12
            roof["frac"] = roof["achieved"] / roof["peak"]
        out[name] = {"trials": T, "launches_timed": OTHER_REPS, "kernel_ms": ms, "node_rounds_per_s": nr / (ms * 1e-3),
                     "trials_per_s": T / (ms * 1e-3), "mean_rounds": rounds / T, "undecided_trials": undecided,
                     "roofline": roof}
        if plan.kernel == benor.BO_KERNEL_MFMA and not (m % 2 == 1 and m > 2 * F):   # KIND 1, 2: deferral chain
            out[name]["kernels_per_launch"] = "matrix-core round 1 + continuation passes + popcount remainder"
        if ms < 1.0:
            # a launch this short is mostly ramp-up: also time 20x the trials for the
            # steady state, SS_REPS such launches back to back (amortising the events)
            h.zero_()
            e0.record(stream)
            for r in range(SS_REPS):
                plan.launch((1 + OTHER_REPS + 20 * r) * T, 20 * T, h.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            ms20 = e0.elapsed_time(e1) / SS_REPS
            nr20, _ = node_rounds(h.cpu().numpy().astype(np.uint64), m, k_max)
            nr20 /= SS_REPS
            out[name]["steady_state"] = {"trials": 20 * T, "launches_timed": SS_REPS, "kernel_ms": ms20,
                                         "node_rounds_per_s": nr20 / (ms20 * 1e-3),
                                         "roofline_frac": roof["frac"] * (nr20 / ms20) / (nr / ms)}
    return out


def delivery_blocks(m, q):
    """Philox4x32-10 blocks one receiver-phase of random delivery draws for its
    q-of-m inbox (oracle_delivery_mask), and the information
    floor log2 C(m, q) / 128.  The sampler's fix-up length is random: its mean
    is taken from the normal approximation of the Bernoulli count."""
    k = min(q, m - q)
    floor = (math.lgamma(m + 1) - math.lgamma(q + 1) - math.lgamma(m - q + 1)) / math.log(2) / 128
    if k >= 64 and 8 * k > m:                          # Bernoulli(a/16) mask + exact fix-up
        a = min(15, max(1, -(-16 * q // m)))
        tz = (a & -a).bit_length() - 1
        mask_words = -(-m // 32) * (4 - tz)
        p = a / 16
        mu, sd = m * p - q, math.sqrt(m * p * (1 - p))
        dist = sd * math.sqrt(2 / math.pi) * math.exp(-mu * mu / (2 * sd * sd)) + mu * math.erf(mu / (sd * math.sqrt(2)))
        accept = (m * p) / m if mu > 0 else 1 - p
        b = max(1, (m - 1).bit_length())
        fields = dist / accept
        return {"sampler": f"bernoulli a={a}/16 + fix-up", "blocks": mask_words / 4 + fields / (32 // b) / 4,
                "floor_blocks": floor}
    return {"sampler": "floyd", "blocks": k / 4, "floor_blocks": floor}


def random_delivery_config(benor, torch, k_max, seed, N=1024, F=341, f=0, T=100_000):
    """SURVEY §8f #4 at N=1024, F=341, f=0 (every receiver tallies a random
    q = N - F of the m = N - f live senders): one warm-up and one timed launch
    at full occupancy, and its real bound -- VALU issue of the Philox blocks
    that draw the delivery masks (41 lane-ops per block), two
    receiver-phases per live node-round -- beside the information floor."""
    import numpy as np

    stream = torch.cuda.current_stream()
    plan = benor.TrialsPlan(N, F, [i < f for i in range(N)], seed=seed, k_max=k_max,
                            mode=benor.BO_MODE_RANDOM_DELIVERY)
    h = torch.zeros(plan.hist_len, dtype=torch.int64, device="cuda")
    plan.launch(0, T // 10, h.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    h.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    plan.launch(T, T, h.data_ptr(), stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    hist = h.cpu().numpy().astype(np.uint64)
    m = plan.live_nodes
    nr, rounds = node_rounds(hist, m, k_max)
    rate = nr / (ms * 1e-3)
    d = delivery_blocks(m, N - F)
    ops = 41 * 2 * d["blocks"]
    return {"trials": T, "launches_timed": 1, "kernel_ms": ms, "node_rounds_per_s": rate, "mean_rounds": rounds / T,
            "agreement_violations": int(hist[-1]),
            "roofline": {"bound": "valu issue (Philox4x32-10 delivery-mask blocks)", "kernel": "random delivery",
                         "sampler": d["sampler"], "philox_blocks_per_node_round": 2 * d["blocks"],
                         "floor_blocks_per_node_round": 2 * d["floor_blocks"], "lane_ops_per_node_round": ops,
                         "unit": "T lane-ops/s", "achieved": rate * ops / 1e12, "peak": SPEC_PEAK_POPC / 1e12,
                         "frac": rate * ops / SPEC_PEAK_POPC,
                         "floor_frac": rate * 41 * 2 * d["floor_blocks"] / SPEC_PEAK_POPC}}


def c5_sweep():
    """BASELINE configs[4] on this GPU: the full C5 phase diagram (N in
    {64..4096} x 32 values of F/N in [0, 0.5), 2^30 trials; benor.cli sweep,
    DESIGN.md §4.5) in this process, wall time from the first plan to the
    read-back, and whether its CSV equals the committed one byte for byte."""
    from benor.cli import grid_cells, rows_csv, run_sweep

    cells = grid_cells([64, 128, 256, 512, 1024, 2048, 4096], 32)
    per_cell = (1 << 30) // len(cells)
    rows, seconds = run_sweep(cells, per_cell, 0x243F6A8885A308D3, 32)
    csv = rows_csv(rows)
    ref = os.path.join(ROOT, "results", "r02_sweep_c5.csv")
    same = os.path.exists(ref) and open(ref).read() == csv
    return {"cells": len(cells), "trials": per_cell * len(cells), "seconds": seconds,
            "trials_per_s": per_cell * len(cells) / seconds, "csv_sha256": hashlib.sha256(csv.encode()).hexdigest()[:16],
            "csv_equals_results_r02_sweep_c5": same}


def event_network(benor, N=1024, F=341, stop_node=500, stop_after=300_000, seed=41):
    """SURVEY §8f #2 at BASELINE configs[3]'s size: one network through the
    reference's calls -- launchNetwork, startConsensus with a mid-run GET /stop
    of one node after `stop_after` deliveries (node.ts:191-194) -- on the
    workgroup-batched event kernel (benor_event_live.hip), as the default
    (live) start runs.  Wall time of startConsensus and the deliveries it
    simulated."""
    m = N - F
    init = [0] * F + [1] * (m // 2) + [0] * (m // 2) + ["?"] * (m % 2)
    faulty = [i < F for i in range(N)]
    out = {}
    for label, sched in (("no stop, sync start (lockstep kernel)", None), ("stop inside round 1", {stop_node: stop_after})):
        benor.launchNetwork(N, F, init, faulty)
        t0 = time.perf_counter()
        benor.startConsensus(N, seed=seed, stop_after=sched, sync=sched is None)
        dt = time.perf_counter() - t0
        st = benor.getNodesState(N)
        out[label] = {"seconds": dt, "stopped_nodes": sum(1 for s in st[F:] if s["killed"])}
    # the default start (bo_consensus_start_live): startConsensus returns at
    # launch, the /stop is sent 1 ms later and lands in the running kernel; the
    # run ends at waitConsensus.  Reported: the wall time from the start to the
    # final states and where the stop landed (replayable as a schedule).
    benor.launchNetwork(N, F, init, faulty)
    t0 = time.perf_counter()
    benor.startConsensus(N, seed=seed)
    t_start = time.perf_counter() - t0
    time.sleep(0.001)                                # the run is under way: the stop lands mid-round
    benor._current.stop_node(stop_node)
    benor.waitConsensus(N)
    st = benor.getNodesState(N)
    dt = time.perf_counter() - t0
    landed = benor._current.live_stop_events()[stop_node]
    out["default (live) start, /stop sent after it"] = {"seconds": dt, "start_returned_after_s": t_start,
                                               "stop_landed_at_delivery": landed,
                                               "stopped_nodes": sum(1 for s in st[F:] if s["killed"])}
    return {"N": N, "F": F, "initial_values": "half 1, half 0, one '?' (every R-phase ties)", **out}


def network_latency(benor, reps=200):
    """BASELINE configs[0]: one start.ts-style network (N=5, F=1, node 4 faulty,
    initial values [1,1,1,0,0], benorconsensus.test.ts:179-223) through the
    reference's own calls -- launchNetwork + startConsensus + getNodesState --
    on the GPU; median and p90 wall time over `reps` networks, for the default
    start (resolves at launch; waitConsensus, then the final states) and the sync one."""
    out = {"networks": reps}
    for label, kw in (("default", {}), ("sync", {"sync": True})):
        times = []
        for rep in range(reps + 5):
            t0 = time.perf_counter()
            benor.launchNetwork(5, 1, [1, 1, 1, 0, 0], [False, False, False, False, True])
            benor.startConsensus(5, seed=rep, **kw)
            benor.waitConsensus(5)
            states = benor.getNodesState(5)
            dt = time.perf_counter() - t0
            if rep >= 5:
                times.append(dt * 1e3)
        times.sort()
        ok = all(s["decided"] and s["x"] == 1 and s["k"] <= 2 for s in states[:4])
        out[label] = {"median_ms": times[len(times) // 2], "p90_ms": times[int(len(times) * 0.9)],
                      "reference_assertions_hold": ok}
    return out


def cpu_baseline(N, F, k_max, seed, budget_s):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    faulty = [i < F for i in range(N)]
    m = N - F

    def timed(nthreads, budget):
        n = 100_000 if nthreads > 1 else 10_000          # calibration sample
        t0 = time.perf_counter()
        oracle.run_trials(N, F, faulty, seed=seed, trial_begin=0, trial_count=n, k_max=k_max, threads=nthreads)
        dt = time.perf_counter() - t0
        n2 = max(n, int(n * budget / max(dt, 1e-6)))
        t0 = time.perf_counter()
        r = oracle.run_trials(N, F, faulty, seed=seed, trial_begin=0, trial_count=n2, k_max=k_max, threads=nthreads)
        dt = time.perf_counter() - t0
        nr, _ = node_rounds(r.hist, m, k_max)
        return nr / dt, n2, dt

    v, n2, dt = timed(threads, budget_s)
    v1, n1, dt1 = timed(1, budget_s * 2 / 3)
    return {"value": v, "unit": "node-rounds/s", "cores": threads, "kind": "port",
            "sample": f"{n2} trials of the bench workload (N={N}, F={F}, k_max={k_max}, same seed), "
                      f"{dt:.1f} s, oracle/benor_oracle.c bit-plane restatement, OpenMP over trials",
            "single_core": {"value": v1, "unit": "node-rounds/s", "cores": 1,
                            "sample": f"{n1} trials, {dt1:.1f} s, same restatement on one thread"}}


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a "
              f"{world}-rank run as {args.gpus} GPUs", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        rank = int(os.environ.get("RANK", "0"))
        line = json.dumps({"dry_run": True, "world": world, "rank": rank, "scaling": args.scaling,
                           "shards": [rank_range(args.scaling, args.warmup + i, rank, world, args.trials)
                                      for i in range(args.steps)]})
        os.write(1, (line + "\n").encode())          # one write: ranks share the pipe
        return

    import numpy as np
    import torch
    import torch.distributed as dist

    import benor
    from benor.parallel import merge_histogram

    env = {k: v for k, v in sorted(os.environ.items()) if k.startswith("BENOR_")}
    forced = sorted(k for k in env if k in benor.KNOBS)
    if forced:
        print(f"bench.py: libbenor knobs set ({', '.join(forced)}): they force kernels, grids or test paths "
              f"(benor.KNOBS); refusing to report a figure for anything but the planner's own choice",
              file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; BENOR_DIST_BACKEND=gloo rehearses several ranks on one GPU
    backend = os.environ.get("BENOR_DIST_BACKEND", "nccl")
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    distributed = env_world is not None          # under a launcher: the collective runs even at world 1
    if distributed:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == world
    N, F, k_max, T = args.N, args.F, args.k_max, args.trials
    faulty = [i < F for i in range(N)]
    plan = benor.TrialsPlan(N, F, faulty, seed=args.seed, k_max=k_max)
    m = plan.live_nodes
    words_per_nr = plan.popc_words_per_node_round
    H = plan.hist_len
    stream = torch.cuda.current_stream()
    hist = torch.zeros(H + 1, dtype=torch.int64, device="cuda")
    # the extra last bin carries 1 per rank: after the all-reduce it counts the
    # ranks whose histograms were merged in that step
    step_hist = torch.zeros(H + 1, dtype=torch.int64, device="cuda")
    one = torch.ones(1, dtype=torch.int64, device="cuda")

    def step(s, ev=None):
        step_hist.zero_()
        step_hist[H:].copy_(one)
        begin, n = rank_range(args.scaling, s, rank, world, T)
        if ev:
            ev[0].record(stream)
        plan.launch(begin, n, step_hist.data_ptr(), stream.cuda_stream)
        if ev:
            ev[1].record(stream)
        merge_histogram(step_hist)              # RCCL merge of the outcome histograms
        hist.add_(step_hist)

    # Clock ramp before the warm-up steps: ~0.3 s of the matrix-core (or
    # popcount) peak probe, whose figure is reported as roofline.peak_probe,
    # then ~0.6 s of a neighbouring shape's kernel (F - 1: the same kernel
    # family and instruction mix under another template instance, so a kernel
    # trace keeps it apart from the bench kernel).  Without the ramp the first
    # two bench launches run 6-15 % slower while clocks and power settle, and a
    # kernel trace of this command averages them in (profiles/r03-v0_summary.md,
    # profiles/r03-v1_summary.md).
    mfma = plan.kernel == benor.BO_KERNEL_MFMA
    peak_measured = None
    if not args.no_peak_probe:
        t_ramp = time.perf_counter()
        while time.perf_counter() - t_ramp < 0.3:
            peak_measured = 2 * benor.mfma_peak(10) if mfma else benor.popc_peak(10)
        if F > 0:
            ramp = benor.TrialsPlan(N, F - 1, [i < F - 1 for i in range(N)], seed=args.seed ^ 0x5A5A, k_max=k_max)
            ramp_hist = torch.zeros(ramp.hist_len, dtype=torch.int64, device="cuda")
            t_ramp = time.perf_counter()
            r = 0
            while time.perf_counter() - t_ramp < 0.6:     # back to back, two launches in flight
                ramp.launch(r * T, T, ramp_hist.data_ptr(), stream.cuda_stream)
                if r:
                    ev_ramp.synchronize()
                ev_ramp = torch.cuda.Event()
                ev_ramp.record(stream)
                r += 1
    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize()
    if not args.no_peak_probe and F > 0:
        del ramp, ramp_hist                      # freed after the warm-up: no hipFree next to a bench launch
    hist.zero_()
    # kernel-only timing with HIP events on the launch stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, ev[i])
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    plan.check()                                   # device-side capacity invariants of the timed launches
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    hh = hist.cpu().numpy().astype(np.uint64)
    h, merged_ranks = hh[:H], int(hh[H])
    assert merged_ranks == world * args.steps, f"histogram merges saw {merged_ranks} rank-steps"
    total_trials = T * args.steps * (1 if args.scaling == "strong" else world)
    assert int(h[:-1].sum()) == total_trials, "histogram lost trials"   # last bin: violations (also counted)
    live_nr, rounds = node_rounds(h, m, k_max)
    value = live_nr / elapsed
    # roofline of the dominant kernel: this rank's launches (rank 0's share of every step)
    my_trials = rank_range(args.scaling, args.warmup, rank, world, T)[1]
    per_launch_nr = live_nr * my_trials / total_trials
    avg_kernel_s = float(np.mean(kern_ms)) * 1e-3
    achieved = per_launch_nr * words_per_nr / avg_kernel_s
    kver = benor.kernel_version()
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):
        try:
            tj = json.load(open(tfile))
            if (tj.get("N"), tj.get("F"), tj.get("trials_per_launch"), tj.get("kernel_version")) == \
                    (N, F, my_trials, kver):
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    per_gpu = "per GPU" if args.scaling == "weak" else "in total"
    out = {
        "metric": METRIC, "value": value, "unit": "node-rounds/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
        "scaling": args.scaling, "vs_baseline": None,
        "dtype": "e2m1 0/1 votes -> f32 exact integer counts" if mfma else "u32",
        "data": "synthetic (Philox initial values)",
        "config": {"workload": f"N={N},F={F} lockstep crash faults, {T} trials {per_gpu} per step, k_max={k_max}",
                   "N": N, "F": F, "live_nodes": m, "trials_per_step": total_trials // args.steps,
                   "trials_per_gpu_per_step": my_trials, "k_max": k_max,
                   "parallelism": f"dp{world} (trial-id sharding, RCCL histogram all-reduce)"},
        "dist": {"world": world, "backend": backend if distributed else None, "ranks_merged_per_step":
                 merged_ranks / args.steps, "hist_sha256": hist_digest(h)},
        "roofline": dict(
            (mfma_roofline(m, per_launch_nr, avg_kernel_s) if mfma else
             {"bound": "valu (v_bcnt_u32_b32 issue)", "achieved": achieved / 1e12, "peak": SPEC_PEAK_POPC / 1e12,
              "unit": "Tpopc/s", "frac": achieved / SPEC_PEAK_POPC, "popc_words_per_node_round": words_per_nr}),
            traffic=traffic, kernel_ms=float(np.mean(kern_ms)),
            peak_probe=(peak_measured / 1e12) if peak_measured else None, kernel_version=kver,
            kernel=benor.KERNEL_NAMES.get(plan.kernel, str(plan.kernel))),
        # BASELINE's metric asks for % of the INT/popcount roofline.  The bench
        # kernel runs on the matrix cores instead, so this states the rate
        # against that ceiling: the v_bcnt issue peak over the popcount words a
        # live node-round needs -- SURVEY §8d's 4*ceil(N/32) (128 at N=1024) and
        # the compact planes' 2 or 3*ceil(m/32) (44 at m=683).
        "int_popcount_ceiling": {
            "peak_popc_words_per_s": SPEC_PEAK_POPC,
            "survey_words_per_node_round": 4 * ((N + 31) // 32),
            "survey_ceiling_node_rounds_per_s": SPEC_PEAK_POPC / (4 * ((N + 31) // 32)),
            "compact_words_per_node_round": words_per_nr,
            "compact_ceiling_node_rounds_per_s": SPEC_PEAK_POPC / words_per_nr,
            "value_over_survey_ceiling": value / (world * SPEC_PEAK_POPC / (4 * ((N + 31) // 32))),
            "value_over_compact_ceiling": value / (world * SPEC_PEAK_POPC / words_per_nr)},
        "all_node_rounds_per_s": rounds * N / elapsed,
        "trials_per_s": total_trials / elapsed,
        "agreement_violations": int(h[-1]),
        "env": env,
    }
    if world == 1 and not args.no_other_configs:
        out["other_configs"] = other_configs(benor, torch, k_max, args.seed)
        out["other_configs"]["C1 N=5,F=1 network API"] = network_latency(benor)
        out["other_configs"]["C4 N=1024,F=341,f=0 random delivery"] = random_delivery_config(benor, torch, k_max, args.seed)
        out["other_configs"]["C4 N=1024,F=341 network API, mid-run /stop"] = event_network(benor)
        out["other_configs"]["C5 sweep (2^30 trials, 224 cells)"] = c5_sweep()
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(N, F, k_max, args.seed, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
