"""Throughput of the round-loop kernels across network shapes (GPU).

For each (N, F, f, mode) -- mode 0 lockstep, 1 random delivery, 2 event level -- runs `trials` trials once for warm-up and once timed
with HIP events on the launch stream, and prints live node-rounds/s and the
popcount-roofline fraction (the plan's algorithmic popcount words per live
node-round -- 2 or 3 * ceil(m/32) lockstep (odd / even vote count), 4 * ceil(m/32)
random delivery -- vs the
v_bcnt issue peak, 39.3 T/s).  One JSON line per shape.

    python tools/perf_matrix.py [--quick]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ben-or-consensus-algorithm_amd"))
PEAK = 256 * 4 * 16 * 2.4e9

SHAPES = [
    # N, F, f (crashed), mode, trials
    (5, 1, 1, 0, 20_000_000), (10, 4, 4, 0, 20_000_000), (10, 5, 5, 0, 2_000_000), (3, 1, 1, 0, 20_000_000),
    (20, 6, 6, 0, 20_000_000), (40, 8, 8, 0, 10_000_000), (48, 20, 20, 0, 10_000_000), (64, 21, 21, 0, 10_000_000),
    (256, 85, 85, 0, 10_000_000), (512, 170, 170, 0, 10_000_000), (1024, 341, 341, 0, 20_000_000),
    (1024, 0, 0, 0, 4_000_000), (1536, 512, 512, 0, 2_000_000), (2048, 682, 682, 0, 1_000_000),
    (4096, 1365, 1365, 0, 400_000), (4096, 0, 0, 0, 100_000),
    # random delivery at full occupancy (>= 8192 resident waves: one trial per wave)
    (10, 4, 2, 1, 2_000_000), (100, 30, 10, 1, 200_000), (1024, 341, 300, 1, 200_000), (1024, 341, 0, 1, 100_000),
    (10, 4, 4, 2, 2_000_000), (32, 10, 10, 2, 200_000), (64, 21, 21, 2, 100_000),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--shapes", default=None, help="'N,F,f,mode,trials;...' instead of the built-in list")
    a = ap.parse_args()
    shapes = SHAPES if not a.shapes else [tuple(int(x) for x in t.split(",")) for t in a.shapes.split(";")]
    import numpy as np
    import torch

    import benor

    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    for (N, F, f, mode, trials) in shapes:
        if a.quick:
            trials = max(1, trials // 10)
        plan = benor.TrialsPlan(N, F, [i < f for i in range(N)], seed=0x1234 + N, k_max=32, mode=mode)
        m = N - f
        h = torch.zeros(plan.hist_len, dtype=torch.int64, device="cuda")
        plan.launch(0, max(1, trials // 10), h.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        h.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        plan.launch(10**9, trials, h.data_ptr(), stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        hist = h.cpu().numpy().astype(np.uint64)
        k = 32
        rounds = sum(r * int(hist[r * 3] + hist[r * 3 + 1] + hist[r * 3 + 2]) for r in range(1, k + 1))
        rounds += k * int(hist[0] + hist[1] + hist[2])
        nr = rounds * m
        words = plan.popc_words_per_node_round
        rate = nr / (ms * 1e-3)
        print(json.dumps({"N": N, "F": F, "f": f, "mode": ["lockstep", "random", "event"][mode], "trials": trials,
                          "mean_rounds": rounds / trials, "ms": round(ms, 3), "node_rounds_per_s": rate,
                          "popc_frac": rate * words / PEAK,
                          "agreement_violations": int(hist[-1]), "kernel_version": benor.kernel_version(),
                          # event level: each live node-round is 2 broadcasts of N messages
                          "messages_per_s": rate * 2 * N if mode == 2 else None}), flush=True)


if __name__ == "__main__":
    main()
