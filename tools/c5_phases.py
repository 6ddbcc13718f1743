"""Where the C5 sweep's wall time goes (GPU): plan creation, launch queueing, GPU
completion, read-back -- for repeated full sweeps in one process (the first one
loads every kernel's code), with the cells round-robin over S streams as
`benor.cli sweep --streams S` does, S alternating over --streams.  With one
stream it also reports per-N GPU time from HIP events on the launch stream.

    python tools/c5_phases.py [--streams 1,4,1,4]    # default sweep: 224 cells, 2^30 trials
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ben-or-consensus-algorithm_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,1")
    a = ap.parse_args()
    import torch

    import benor

    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    Ns = [64, 128, 256, 512, 1024, 2048, 4096]
    steps, seed, k_max = 32, 0x243F6A8885A308D3, 32   # the sweep defaults (benor.cli)
    cells = [(N, int(i * 0.5 / steps * N)) for N in Ns for i in range(steps)]
    per_cell = (1 << 30) // len(cells)
    for rep, S in enumerate(int(x) for x in a.streams.split(",")):
        t0 = time.perf_counter()
        plans = [benor.TrialsPlan(N, F, seed=seed ^ (N << 20) ^ F, k_max=k_max) for (N, F) in cells]
        t1 = time.perf_counter()
        hists = torch.zeros((len(cells), plans[0].hist_len), dtype=torch.int64, device="cuda")
        ev = {}
        streams = [st] + [torch.cuda.Stream() for _ in range(S - 1)]
        for s in streams[1:]:
            s.wait_stream(st)
        for ci, plan in enumerate(plans):
            N = cells[ci][0]
            if S == 1 and N not in ev:
                ev[N] = [torch.cuda.Event(enable_timing=True), None]
                ev[N][0].record(st)
            plan.launch(0, per_cell, hists[ci].data_ptr(), streams[ci % S].cuda_stream)
            if S == 1 and (ci + 1 == len(cells) or cells[ci + 1][0] != N):
                ev[N][1] = torch.cuda.Event(enable_timing=True)
                ev[N][1].record(st)
        for s in streams[1:]:
            st.wait_stream(s)
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        h = hists.cpu()
        t4 = time.perf_counter()
        print(json.dumps({"sweep": rep, "streams": S, "cells": len(cells), "per_cell": per_cell,
                          "plans_s": t1 - t0, "queue_s": t2 - t1, "drain_s": t3 - t2, "readback_s": t4 - t3,
                          "total_s": t4 - t0, "checksum": int(h.sum()), "digest": int((h * torch.arange(1, h.numel() + 1).view_as(h)).sum()),
                          "gpu_ms_per_N": {N: round(e[0].elapsed_time(e[1]), 3) for N, e in ev.items()}}), flush=True)
        del plans


if __name__ == "__main__":
    main()
