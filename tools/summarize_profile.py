"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>/) into profiles/.

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_valu_probe.txt     VALU issue-rate probe output (copied)
  profiles/<tag>_summary.md         PMC counters per launch of the lockstep kernel, derived rates
  profiles/pmc_traffic.json         HBM bytes per launch (bench.py reads it for roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7:
FETCH_SIZE and WRITE_SIZE (KiB) come from separate --pmc passes; on gfx950
FETCH_SIZE reads half the bytes of a wide coalesced stream, so it is doubled
(an upper bound for this kernel's few narrow reads); WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


KERNELS = ("lockstep", "mfma")   # the bench shape's kernel: popcount (lockstep_*) or matrix core (mfma_*)


def pmc_per_dispatch(path, kernel_subs=KERNELS):
    agg = defaultdict(list)
    meta = {}
    for f in glob.glob(os.path.join(path, "pmc*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if not any(k in r["Kernel_Name"] for k in kernel_subs):
                continue
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                      "VGPR_Count", "SGPR_Count", "Scratch_Size")}
    return {k: sum(v) / len(v) for k, v in agg.items()}, meta


def main(tag, trials, N=1024, F=341):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
    probe = os.path.join(src, "valu_probe.txt")
    if os.path.exists(probe):
        shutil.copy(probe, os.path.join(dst, f"{tag}_valu_probe.txt"))
    c, meta = pmc_per_dispatch(src)
    m = N - F
    kname = meta.get("Kernel_Name", "")
    lines = [f"# Profile {tag}: {'matrix-core' if 'mfma' in kname else 'lockstep'} kernel, N={N}, F={F}, "
             f"{trials} trials per launch", ""]
    lines += [f"- {k}: {v}" for k, v in meta.items()]
    lines += ["", "| counter | per launch | per trial |", "|---|---|---|"]
    for k in sorted(c):
        lines.append(f"| {k} | {c[k]:.6g} | {c[k] / trials:.4g} |")
    if "SQ_INSTS_VALU" in c and "mfma" in kname:
        W = (m + 63) // 64
        MT = 2 * W - (1 if m <= 64 * (W - 1) + 32 else 0)   # 32-receiver tiles (benor_mfma.h)
        KP = (MT + 1) // 2
        mfma = (MT * W + MT * KP) / 32.0                      # R-phase MT x W, P-phase MT x KP, per 32 trials
        lines += ["", f"- MFMA (32x32x64 e2m1) per trial: {mfma:.2f} (R-phase {MT}x{W} + P-phase {MT}x{KP} per 32 trials)",
                  f"- VALU instructions per trial (SQ_INSTS_VALU, MFMA included): {c['SQ_INSTS_VALU'] / trials:.1f} "
                  f"(non-MFMA: {c['SQ_INSTS_VALU'] / trials - mfma:.1f})"]
    elif "SQ_INSTS_VALU" in c:
        W = (m + 63) // 64
        per = 4 if m % 2 else 6   # words per receiver group / W: 2 (R-phase c1) + 2 (P c1, odd m) or 4 (P c0, c1)
        bcnt = per * W * W
        lines += ["", f"- v_bcnt per trial (one round; {per}W words per receiver group x W groups, W = ceil(m/64)): {bcnt}",
                  f"- VALU instructions per trial: {c['SQ_INSTS_VALU'] / trials:.1f} "
                  f"(non-v_bcnt: {c['SQ_INSTS_VALU'] / trials - bcnt:.1f})"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0          # GRBM counts per XCD; 8 XCDs
        simd_cycles = cyc * 1024.0                # 256 CU x 4 SIMD
        lines += [f"- kernel cycles (GRBM_GUI_ACTIVE / 8 XCDs): {cyc:.4g}",
                  f"- matrix-core busy: {c['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles:.3f} of SIMD-cycles "
                  f"(SQ_VALU_MFMA_BUSY_CYCLES = 32 x SQ_INSTS_MFMA: "
                  f"{c['SQ_VALU_MFMA_BUSY_CYCLES'] / max(1.0, c.get('SQ_INSTS_MFMA', 0.0)):.1f} per instruction)",
                  f"- VALU co-executing with the matrix core: {c.get('SQ_VALU_MFMA_COEXEC_CYCLES', 0.0) / simd_cycles:.3f} "
                  f"of SIMD-cycles ({c.get('SQ_VALU_MFMA_COEXEC_CYCLES', 0.0) / c['SQ_VALU_MFMA_BUSY_CYCLES']:.3f} "
                  f"of the busy cycles)"]
    if "GRBM_GUI_ACTIVE" in c and stats:
        for r in csv.DictReader(open(stats[0])):
            if any(k in r["Name"] for k in KERNELS):
                avg_ns = float(r["AverageNs"])
                lines.append(f"- kernel-trace average duration (bench launches): {avg_ns / 1e6:.3f} ms")
    hbm = None
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        hbm = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
        lines.append(f"- HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, KiB -> B): {hbm:.0f}")
        kver = None                  # kernel-source digest printed by the profiled bench run
        for log in sorted(glob.glob(os.path.join(src, "pmc*.log"))):
            for line in open(log):
                if line.startswith("{"):
                    try:
                        kver = json.loads(line)["roofline"]["kernel_version"]
                    except (ValueError, KeyError):
                        pass
        if (N, F) == (1024, 341):   # bench.py reads the bench shape's traffic only
            json.dump({"N": N, "F": F, "trials_per_launch": trials, "kernel_version": kver,
                       "hbm_bytes_per_launch": hbm,
                       "fetch_kib": c["FETCH_SIZE"], "write_kib": c["WRITE_SIZE"],
                       "source": f"profiles/{tag}_summary.md"},
                      open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    open(os.path.join(dst, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1].startswith("-"):
        sys.exit(__doc__ + "\nusage: python tools/summarize_profile.py <tag> [trials] [N F]")
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000,
         *(int(x) for x in sys.argv[3:5]))
