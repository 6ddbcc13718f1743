"""CPU baseline per BASELINE config: the oracle's bit-plane
restatement (oracle/benor_oracle.c, a port -- the reference's Express network
cannot run here) timed on one thread and on every host thread
(OMP_NUM_THREADS, 16 on the GPU box), live node-rounds/s, one JSON line per
config.  Test infrastructure: it times the checker, never the product.

    python tools/cpu_baseline_table.py [--seconds S]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

CONFIGS = [("C1 N=5,F=1", 5, 1), ("C2 N=10,F=4", 10, 4), ("C2 N=10,F=5", 10, 5), ("C3 N=256,F=85", 256, 85),
           ("C4 N=1024,F=341", 1024, 341)]


def rate(N, F, threads, budget, k_max=16, seed=0x243F6A8885A308D3):
    import oracle
    from bench import node_rounds

    fl = [i < F for i in range(N)]
    n = 2000
    while True:
        t0 = time.perf_counter()
        r = oracle.run_trials(N, F, fl, seed=seed, trial_begin=0, trial_count=n, k_max=k_max, threads=threads)
        dt = time.perf_counter() - t0
        if dt > budget / 4 or n >= 1 << 30:
            break
        n *= 4
    nr, _ = node_rounds(r.hist, N - F, k_max)
    return nr / dt, n, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=4.0)
    a = ap.parse_args()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    for name, N, F in CONFIGS:
        r1, n1, d1 = rate(N, F, 1, a.seconds)
        ra, na, da = rate(N, F, threads, a.seconds)
        print(json.dumps({"config": name, "N": N, "F": F, "k_max": 16, "one_core": r1, "one_core_sample": [n1, d1],
                          "all_cores": ra, "cores": threads, "all_cores_sample": [na, da],
                          "unit": "live node-rounds/s"}), flush=True)


if __name__ == "__main__":
    main()
