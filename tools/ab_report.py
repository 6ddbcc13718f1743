"""Summarise gpurun_out/ab.jsonl (tools/ab.sh): best ms per (lib, shape) and speedup vs the first lib."""
import json
import sys
from collections import defaultdict

best = defaultdict(lambda: float("inf"))
frac = {}
libs = []
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.jsonl"):
    d = json.loads(line)
    if d["lib"] not in libs:
        libs.append(d["lib"])
    key = (d["lib"], d["N"], d["F"], d["f"], d["mode"])
    if d["ms"] < best[key]:
        best[key] = d["ms"]
        frac[key] = d["popc_frac"]
for shape in sorted({k[1:] for k in best}):
    b = best[(libs[0],) + shape]
    cols = "  ".join(f"{lib} {best[(lib,) + shape]:8.3f} ms ({frac[(lib,) + shape]:.3f}) x{b / best[(lib,) + shape]:.3f}"
                     for lib in libs if (lib,) + shape in best)
    print(f"N={shape[0]:5d} F={shape[1]:5d} f={shape[2]:5d} {shape[3]:9s} {cols}")
