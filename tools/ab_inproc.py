"""Interleaved A/B of environment-selected variants in ONE process (GPU).

The runtime reads its A/B knobs (BENOR_BIG_FORM, BENOR_COOP_BW, BENOR_BLOCKS_PER_CU,
... -- the registered ones, benor.KNOBS; any other variable is refused, since a
removed knob would time two identical variants) at every launch, so variants can
alternate launch by launch on one plan, one process, one box: ROUNDS rounds,
each timing every variant once per shape in rotated order (cdna_hip_programming.md
section 5.4 rule 24).  Each timing is REPS back-to-back launches between HIP
events on the launch stream.  Prints one JSON line per (shape, variant) with the
median and minimum ms per launch and the variant's median / first variant's.

    python tools/ab_inproc.py --variants "coop=BENOR_BIG_FORM:coop;wave=BENOR_BIG_FORM:wave" \
        --shapes "4096,1365,400000;4096,0,100000" [--rounds 7] [--reps 3]

A shape may carry a fourth field f < F (the first f nodes crashed, the rest of
F the random-delivery slack: BO_MODE_RANDOM_DELIVERY).  Every line also reports
the live node-rounds per second its launches represent (bench.py node_rounds),
so variants that change the outcome (a diagnostic cap) compare per unit of work.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ben-or-consensus-algorithm_amd"))


def parse_variants(spec):
    out = []
    for item in spec.split(";"):
        name, _, kv = item.partition("=")
        env = {}
        for pair in filter(None, kv.split(",")):
            k, _, v = pair.partition(":")
            env[k] = v
        out.append((name, env))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True, help="'name=VAR:val,VAR:val;name2=...' ('name=' = no variables)")
    ap.add_argument("--shapes", required=True,
                    help="'N,F,trials[,f];...' (the first f nodes crashed, f = F by default)")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    variants = parse_variants(a.variants)
    shapes = []
    for sp in a.shapes.split(";"):
        v = [int(x) for x in sp.split(",")]
        shapes.append((v[0], v[1], v[2], v[3] if len(v) > 3 else v[1]))
    knobs = sorted({k for _, env in variants for k in env})

    import benor
    unknown = [k for k in knobs if k not in benor.KNOBS]
    if unknown:
        ap.error(f"not a registered libbenor knob (benor.KNOBS): {unknown}")

    import numpy as np
    import torch

    sys.path.insert(0, ROOT)
    from bench import node_rounds

    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()

    def set_env(env):
        for k in knobs:
            os.environ.pop(k, None)
        os.environ.update(env)

    times, work = {}, {}
    for N, F, T, f in shapes:
        mode = benor.BO_MODE_RANDOM_DELIVERY if f < F else benor.BO_MODE_LOCKSTEP
        plan = benor.TrialsPlan(N, F, [i < f for i in range(N)], seed=0x5EED + N, k_max=32, mode=mode)
        h = torch.zeros(plan.hist_len, dtype=torch.int64, device="cuda")
        for _, env in variants:                       # warm-up per variant (allocations, code load)
            set_env(env)
            plan.launch(0, max(1, T // 10), h.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        nxt = T
        for rnd in range(a.rounds):
            order = variants[rnd % len(variants):] + variants[:rnd % len(variants)]
            for name, env in order:
                set_env(env)
                h.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(a.reps):
                    plan.launch(nxt, T, h.data_ptr(), st.cuda_stream)
                    nxt += T
                e1.record(st)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                times.setdefault((N, F, T, f, name), []).append(ms)
                nr, _ = node_rounds(h.cpu().numpy().astype(np.uint64), N - f, 32)
                work.setdefault((N, F, T, f, name), []).append(nr / a.reps / (ms * 1e-3))
    set_env({})
    for N, F, T, f in shapes:
        base = statistics.median(times[(N, F, T, f, variants[0][0])])
        for name, _ in variants:
            t = times[(N, F, T, f, name)]
            print(json.dumps({"N": N, "F": F, "f": f, "trials": T, "variant": name, "median_ms": statistics.median(t),
                              "min_ms": min(t), "rounds": len(t), "median_vs_first": statistics.median(t) / base,
                              "node_rounds_per_s": statistics.median(work[(N, F, T, f, name)]),
                              "kernel_version": benor.kernel_version()}), flush=True)


if __name__ == "__main__":
    main()
