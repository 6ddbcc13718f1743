"""Summarise one tools/gpu.sh session (gpurun_out/<TAG>/) into profiles/<TAG>_*.

    python tools/pmc_report.py <TAG>

Writes
  profiles/<TAG>_kernel_stats.csv  rocprofv3 --kernel-trace --stats of the bench command (copied)
  profiles/<TAG>_bench.json        the bench line printed by that same traced run
  profiles/<TAG>_summary.md        (1) reconciliation: for the headline and every other_configs
                                   entry, the kernel's trace durations beside the line's HIP-event
                                   kernel_ms and the roofline fraction recomputed from the trace;
                                   (2) per shape (pmc_<shape>/), the PMC counters of the timed launch
                                   (the last dispatch of the shape's kernel) per launch and per trial,
                                   with derived busy fractions and HBM bytes.

HBM bytes follow MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE (KiB)
from separate --pmc passes, FETCH_SIZE doubled on gfx950 (it counts half the bytes of
a wide coalesced stream; an upper bound for these kernels' narrow reads).
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 256 * 4
XCDS = 8


def last_dispatch(path):
    """Counters of the timed launch's main kernel.  perf_matrix runs a warm-up
    launch (a tenth of the trials, possibly on another kernel), then the timed
    one, and a deferral shape's launch is several kernels (round 1, continuation
    passes, popcount remainder).  Every pass replays the same dispatch sequence,
    so the launch is chosen once, as the longest dispatch (GRBM_GUI_ACTIVE) of
    the pass that counts it, and taken at the same position in every pass."""
    passes = []
    for f in sorted(glob.glob(os.path.join(path, "p*", "*counter_collection.csv"))):
        rows = [r for r in csv.DictReader(open(f)) if "benor::" in r["Kernel_Name"] and "peak" not in r["Kernel_Name"]]
        if rows:
            ids = sorted({int(r["Dispatch_Id"]) for r in rows})
            passes.append((rows, ids))
    pick = None
    for rows, ids in passes:
        dur = defaultdict(float)
        for r in rows:
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                dur[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        if dur:
            pick = ids.index(max(dur, key=lambda i: (dur[i], i)))
            break
    per, meta = {}, {}
    for rows, ids in passes:
        want = ids[pick] if pick is not None and pick < len(ids) else ids[-1]
        agg = defaultdict(float)
        for r in rows:
            if int(r["Dispatch_Id"]) == want:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                          "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size")}
        for k, v in agg.items():
            per.setdefault(k, v)          # a counter measured in two passes: keep the first
    return per, meta


def shape_of(path):
    for log in glob.glob(os.path.join(path, "p*.log")):
        for line in open(log):
            if line.startswith("{"):
                return json.loads(line)
    return None


def trace_durations(tag_dir):
    """Per kernel name: (first dispatch id, durations in ms of its launches in dispatch order)."""
    out = defaultdict(list)
    for f in glob.glob(os.path.join(tag_dir, "trace", "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            out[r["Kernel_Name"]].append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    return {k: (min(v)[0], [d for _, d in sorted(v)]) for k, v in out.items()}


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    lines = [f"# Profile {tag}", "", f"Source: `tools/gpu.sh` session `{tag}` on one MI355X; summarised by "
             f"`tools/pmc_report.py {tag}`.", ""]
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
    bench = None
    if stats:
        shutil.copy(stats[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
        for line in open(os.path.join(src, "trace_bench.log")):
            if line.startswith("{"):
                bench = json.loads(line)
        if bench:
            json.dump(bench, open(os.path.join(dst, f"{tag}_bench.json"), "w"), indent=1)
        durs = trace_durations(src)
        lines += ["## Bench line vs kernel trace (same traced run)", "",
                  f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py {bench_args()}`.  The bench "
                  "kernel's launches are the warm-up steps followed by the timed steps; other_configs launch "
                  "once (warm-up), then OTHER_REPS back to back, then once more at 20x the trials "
                  "(steady state).", "",
                  "| entry | kernel | trace launches | trace avg ms (timed launches) | line kernel_ms | "
                  "line frac | frac from trace | ratio |", "|---|---|---|---|---|---|---|---|"]
        if bench:
            lines += reconcile(bench, durs)
            lines += ["", f"- line `ms_per_step` {bench['ms_per_step']:.4f} ms; bench-kernel trace average over "
                          f"every launch (stats CSV) {stats_avg(stats[0], bench_kernel(durs, bench, bench['steps'])):.4f} ms", ""]
    for d in sorted(glob.glob(os.path.join(src, "pmc_*"))):
        c, meta = last_dispatch(d)
        shp = shape_of(d) or {}
        if not c:
            continue
        trials = shp.get("trials", 1)
        lines += [f"## PMC `{os.path.basename(d)[4:]}`: N={shp.get('N')}, F={shp.get('F')}, f={shp.get('f')}, "
                  f"{shp.get('mode')}, {trials} trials (timed launch of tools/perf_matrix.py)", ""]
        lines += [f"- {k}: {v}" for k, v in meta.items()]
        lines += [f"- perf_matrix line (same run, pass 1): {json.dumps(shp)}", "",
                  "| counter | per launch | per trial |", "|---|---|---|"]
        for k in sorted(c):
            lines.append(f"| {k} | {c[k]:.6g} | {c[k] / trials:.4g} |")
        lines.append("")
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        if cyc:
            lines.append(f"- kernel cycles (GRBM_GUI_ACTIVE / {XCDS} XCDs): {cyc:.6g} "
                         f"({cyc / 2.4e3:.2f} us at 2.4 GHz)")
        if "SQ_INSTS_VALU" in c:
            v = c["SQ_INSTS_VALU"]
            mf = c.get("SQ_INSTS_MFMA", 0.0)
            lines.append(f"- wave-level VALU instructions per trial: {v / trials:.3f} (MFMA {mf / trials:.3f}, "
                         f"other {(v - mf) / trials:.3f}); lane-level: {64 * (v - mf) / trials:.1f} non-MFMA lane-ops")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and cyc:
            lines.append(f"- matrix core busy: SQ_VALU_MFMA_BUSY_CYCLES / (cycles x {SIMDS} SIMDs) = "
                         f"{c['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * SIMDS):.3f}; VALU co-executing: "
                         f"{c.get('SQ_VALU_MFMA_COEXEC_CYCLES', 0.0) / (cyc * SIMDS):.3f}")
        if "SQ_LDS_BANK_CONFLICT" in c and "SQ_INSTS_LDS" in c and c["SQ_INSTS_LDS"]:
            lines.append(f"- LDS: {c['SQ_INSTS_LDS'] / trials:.4f} instructions per trial, "
                         f"{c['SQ_LDS_BANK_CONFLICT'] / trials:.4f} bank-conflict cycles per trial "
                         f"({c['SQ_LDS_BANK_CONFLICT'] / c['SQ_INSTS_LDS']:.3f} per LDS instruction)")
        if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            lines.append(f"- waves waiting on any instruction: {c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f} "
                         f"of wave-cycles (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES)")
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            hbm = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
            lines.append(f"- HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE): {hbm:.0f} "
                         f"({hbm / trials:.4f} per trial)")
            if (shp.get("N"), shp.get("F"), shp.get("f"), shp.get("mode")) == (1024, 341, 341, "lockstep"):
                # bench.py quotes roofline.traffic from here when the kernel digest matches
                json.dump({"N": 1024, "F": 341, "trials_per_launch": trials,
                           "kernel_version": shp.get("kernel_version"), "hbm_bytes_per_launch": hbm,
                           "fetch_kib": c["FETCH_SIZE"], "write_kib": c["WRITE_SIZE"],
                           "source": f"profiles/{tag}_summary.md"},
                          open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
        lines.append("")
    open(os.path.join(dst, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


def bench_args():
    return os.environ.get("BENCH_ARGS", "--steps 20 --warmup 5")


def bench_kernel(durs, bench=None, steps=None):
    """The headline kernel: with the bench line, the kernel whose last `steps`
    launches average closest to the line's kernel_ms (the clock-ramp shape run
    before the warm-up can hold more total time); else the most total time."""
    if bench and steps:
        want = bench["roofline"]["kernel_ms"]
        cand = [k for k in durs if "benor::" in k and len(durs[k][1]) >= steps]
        if cand:
            return min(cand, key=lambda k: abs(statistics.mean(durs[k][1][-steps:]) - want))
    return max(durs, key=lambda k: sum(durs[k][1]))


def stats_avg(path, name):
    for r in csv.DictReader(open(path)):
        if r["Name"] == name:
            return float(r["AverageNs"]) / 1e6
    return float("nan")


def reconcile(bench, durs):
    """Rows of the reconciliation table.  The headline kernel: its last `steps`
    launches are the timed ones.  other_configs run in order, each on its own
    kernel: one warm-up launch, `launches_timed` timed ones, then the steady-state
    launch; they are matched to the benor kernels first dispatched after the
    headline's launches, in dispatch order."""
    rows = []
    steps = bench["steps"]
    bk = bench_kernel(durs, bench, steps)
    timed = durs[bk][1][-steps:]
    avg = statistics.mean(timed)
    rf = bench["roofline"]
    rows.append(f"| headline | `{short(bk)}` | {len(durs[bk][1])} | {avg:.4f} | {rf['kernel_ms']:.4f} | "
                f"{rf['frac']:.4f} | {rf['frac'] * rf['kernel_ms'] / avg:.4f} | {rf['kernel_ms'] / avg:.3f} |")
    # each config's kernel: the first unused benor kernel of its family
    # (the roofline's "kernel" name) dispatched after the headline
    later = sorted((v[0], k) for k, v in durs.items()
                   if k != bk and "benor::" in k and "peak" not in k and v[0] > durs[bk][0])
    used = set()
    for name, oc in bench.get("other_configs", {}).items():
        if "kernel_ms" not in oc or "kernels_per_launch" in oc:   # several kernels per plan launch: no 1:1 match
            continue
        fam = family_symbol(oc.get("roofline", {}).get("kernel", ""))
        cand = [k for _, k in later if k not in used and (fam is None or fam in k)]
        if not cand:
            continue
        k = cand[0]
        used.add(k)
        reps = oc.get("launches_timed", 10)
        d = durs[k][1]
        a = statistics.mean(d[1:1 + reps])
        fr = oc["roofline"]["frac"]
        rows.append(f"| {name} | `{short(k)}` | {reps} of {len(d)} (#1..#{reps}) | {a:.5f} | "
                    f"{oc['kernel_ms']:.5f} | {fr:.4f} | {fr * oc['kernel_ms'] / a:.4f} | {oc['kernel_ms'] / a:.3f} |")
        ss = oc.get("steady_state")
        sreps = ss.get("launches_timed", 1) if ss else 0
        if ss and len(d) >= 1 + reps + sreps:
            a2 = statistics.mean(d[1 + reps:1 + reps + sreps])
            rows.append(f"| {name}, steady state ({ss['trials']} trials) | `{short(k)}` | {sreps} (#{1 + reps}..#{reps + sreps}) "
                        f"| {a2:.5f} | {ss['kernel_ms']:.5f} | {ss['roofline_frac']:.4f} | "
                        f"{ss['roofline_frac'] * ss['kernel_ms'] / a2:.4f} | {ss['kernel_ms'] / a2:.3f} |")
    return rows


def family_symbol(kernel_name):
    """Kernel-symbol substring of a roofline's kernel family (benor.KERNEL_NAMES)."""
    for fam, sym in (("packed matrix core", "benor_mfma_small_kernel"), ("random delivery", "benor_random_kernel"),
                     ("matrix core", "benor_mfma_"), ("lane", "benor_lane_kernel"), ("W popcount", "_w_kernel"),
                     ("blocked", "blocked_kernel"), ("event", "benor_event_kernel")):
        if fam in kernel_name:
            return sym
    return None


def short(k):
    return k.replace("void benor::", "").replace("(benor::KParams)", "")


if __name__ == "__main__":
    if len(sys.argv) != 2:
        sys.exit(__doc__)
    main(sys.argv[1])
