"""Per-basic-block instruction mix of one kernel in a hipcc --save-temps .s file.

usage: python tools/isa_blocks.py <file.s> <kernel-symbol-substring> [--min-valu N]
Prints each block (label, loop depth comment) with its VALU / SALU / LDS /
readlane-writelane counts, so the hot path's non-popcount VALU can be read
off without a GPU.  Inspection only.
"""
import re
import sys
from collections import Counter


def blocks(path, sym):
    lines = open(path).read().split("\n")
    # the function's label line: "<mangled name>:" (optionally followed by a comment)
    start = next(i for i, l in enumerate(lines)
                 if l.startswith("_Z") and sym in l.split(":", 1)[0] and ":" in l)
    cur, out = "entry", []
    cnt = Counter()
    for l in lines[start + 1:]:
        if l.strip().startswith("s_endpgm"):
            break
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):?", l)
        if m:
            out.append((cur, cnt))
            cur, cnt = (m.group(1) + "  " + l.split(";", 1)[-1].strip() if l.startswith(".") else m.group(1)), Counter()
            continue
        t = l.strip().split()
        if not t or t[0].startswith(";") or t[0].startswith("."):
            continue
        op = t[0]
        if op.startswith("v_bcnt"):
            cnt["bcnt"] += 1
        elif op.startswith("v_readlane") or op.startswith("v_writelane"):
            cnt["rl/wl"] += 1
        elif op.startswith("v_"):
            cnt["valu"] += 1
        elif op.startswith("s_nop"):
            cnt["nop"] += 1
        elif op.startswith("s_"):
            cnt["salu"] += 1
        elif op.startswith("ds_"):
            cnt["lds"] += 1
        elif op.startswith("global_") or op.startswith("buffer_"):
            cnt["vmem"] += 1
    out.append((cur, cnt))
    return out


if __name__ == "__main__":
    path, sym = sys.argv[1], sys.argv[2]
    for name, c in blocks(path, sym):
        if sum(c.values()):
            print(f"{name[:90]:90s} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
