"""Summarise gpurun_out/ab.jsonl (tools/ab.sh): best ms per (lib, shape) and new/base speedup."""
import json
import sys
from collections import defaultdict

best = defaultdict(lambda: float("inf"))
frac = {}
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.jsonl"):
    d = json.loads(line)
    key = (d["N"], d["F"], d["f"], d["mode"])
    if d["ms"] < best[(d["lib"],) + key]:
        best[(d["lib"],) + key] = d["ms"]
        frac[(d["lib"],) + key] = d["popc_frac"]
for key in sorted({k[1:] for k in best}):
    b, n = best[("base",) + key], best[("new",) + key]
    print(f"N={key[0]:5d} F={key[1]:5d} f={key[2]:5d} {key[3]:9s} base {b:8.3f} ms ({frac[('base',) + key]:.3f})"
          f"  new {n:8.3f} ms ({frac[('new',) + key]:.3f})  speedup {b / n:.3f}")
