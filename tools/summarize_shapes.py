"""Summarise tools/prof_r02_shapes.sh output into profiles/ (per-shape PMC of the
timed launch -- the last dispatch of each pass -- with derived per-trial rates).

    python tools/summarize_shapes.py r02
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = {"lane10": ("lane", 20_000_000, "N=10, F=4 lockstep (lane kernel, BASELINE configs[1])"),
          "n256": ("lockstep_w", 10_000_000, "N=256, F=85 lockstep (W kernel, W=3, BASELINE configs[2])"),
          "rd1024": ("random", 100_000, "N=1024, F=341, f=0 random delivery (Bernoulli + fix-up sampler)")}


def last_dispatch(path, sub):
    per = defaultdict(dict)
    for f in glob.glob(os.path.join(path, "pmc*", "*counter_collection.csv")):
        rows = [r for r in csv.DictReader(open(f)) if sub in r["Kernel_Name"]]
        if not rows:
            continue
        last = max(int(r["Dispatch_Id"]) for r in rows)
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                per[r["Counter_Name"]] = float(r["Counter_Value"])
                per["_kernel"] = r["Kernel_Name"]
    return per


def main(tag):
    src = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(src, f"prof_{tag}_trace", "shapes_kernel_stats.csv"),
                os.path.join(dst, f"{tag}-shapes_kernel_stats.csv"))
    shutil.copy(os.path.join(src, f"prof_{tag}_trace", "pm.jsonl"), os.path.join(dst, f"{tag}-shapes_perf.jsonl"))
    for key, (sub, trials, what) in SHAPES.items():
        c = last_dispatch(os.path.join(src, f"prof_{tag}-{key}"), sub)
        if not c:
            continue
        lines = [f"# Profile {tag}-{key}: {what}, {trials} trials per launch", "",
                 "Source: `tools/prof_r02_shapes.sh` (`tools/prof_shape.sh` PMC passes over `tools/perf_matrix.py`);",
                 "the timed launch (last dispatch of each pass) only.", "", f"- Kernel_Name: {c.pop('_kernel')}", "",
                 "| counter | per launch | per trial |", "|---|---|---|"]
        for k in sorted(c):
            lines.append(f"| {k} | {c[k]:.6g} | {c[k] / trials:.4g} |")
        if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
            # GRBM_GUI_ACTIVE sums the 8 XCDs; VALU busy = VALU issue cycles / SIMD cycles
            cycles = c["GRBM_GUI_ACTIVE"] / 8.0
            busy = c["SQ_INSTS_VALU"] * 4.17 / 1024.0 / cycles
            lines += ["", f"- VALU instructions per trial: {c['SQ_INSTS_VALU'] / trials:.1f}",
                      f"- kernel cycles (GRBM_GUI_ACTIVE / 8 XCDs): {cycles:.4g}; VALU issue ~{busy:.0%} busy "
                      f"(at 4.17 cycles per wave64 instruction over 1024 SIMDs)"]
        open(os.path.join(dst, f"{tag}-{key}_summary.md"), "w").write("\n".join(lines) + "\n")
        print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
