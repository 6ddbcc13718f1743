"""Kernel time of one plan's launches, averaged over 10 back-to-back launches
(HIP events around the burst; the plan's own grid choice).  One JSON line per
shape:  python tools/burst_time.py "N,F,trials;..." """
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
    for spec in sys.argv[1].split(";"):
        N, F, T = (int(x) for x in spec.split(","))
        plan = benor.TrialsPlan(N, F, [i < F for i in range(N)], seed=7, k_max=16)
        h = torch.zeros(plan.hist_len, dtype=torch.int64, device="cuda")
        plan.launch(0, T, h.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for r in range(10):
            plan.launch((r + 1) * T, T, h.data_ptr(), st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        print(json.dumps({"N": N, "F": F, "trials": T, "kernel": plan.kernel, "us": e0.elapsed_time(e1) / 10 * 1e3}),
              flush=True)


if __name__ == "__main__":
    main()
