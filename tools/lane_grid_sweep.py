"""Kernel time of short launches vs grid size (BENOR_BLOCKS_PER_CU): one JSON
line per (shape, trials, blocks per CU), the average of 10 back-to-back
launches timed with HIP events."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ben-or-consensus-algorithm_amd"))


def main():
    import torch

    import benor

    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    shapes = [(10, 4), (5, 1), (20, 6), (64, 21)]
    for N, F in shapes:
        plan = benor.TrialsPlan(N, F, [i < F for i in range(N)], seed=7, k_max=16)
        h = torch.zeros(plan.hist_len, dtype=torch.int64, device="cuda")
        for T in (10**6, 3 * 10**6, 10**7):
            for bpc in (8, 6, 4, 3, 2, 1):
                os.environ["BENOR_BLOCKS_PER_CU"] = str(bpc)
                plan.launch(0, T, h.data_ptr(), st.cuda_stream)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for r in range(10):
                    plan.launch((r + 1) * T, T, h.data_ptr(), st.cuda_stream)
                e1.record(st)
                torch.cuda.synchronize()
                print(json.dumps({"N": N, "F": F, "trials": T, "blocks_per_cu": bpc, "kernel": plan.kernel,
                                  "us": e0.elapsed_time(e1) / 10 * 1e3}), flush=True)


if __name__ == "__main__":
    main()
