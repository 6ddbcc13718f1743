"""Documentation drift: every repo path the docs cite exists.

The docs cite profiles, tools, sources and tests by path; a renamed or deleted
file leaves a dangling reference that no other test sees.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "ben-or-consensus-algorithm_amd"
DOCS = ["DESIGN.md", "README.md", "BASELINE.md", "INTEGRATION.md", "profiles/README.md"]
# a backquoted path under one of the repo's own top-level directories
CITED = re.compile(r"`((?:profiles|tools|tests|oracle|include|csrc|js|benor|results)/[^`\s:]+)")


def cited_paths(doc):
    text = open(os.path.join(ROOT, doc), encoding="utf-8").read()
    out = set()
    for m in CITED.finditer(text):
        p = m.group(1).rstrip(".")
        p = p.split("::")[0]
        if any(c in p for c in "*<>{}") or p.endswith("/"):
            continue                                   # globs, templates, directories
        out.add(p)
    return sorted(out)


# r01-r03's one-off GPU wrappers, folded into tools/gpu.sh (profiles/README.md
# says so); DESIGN.md still names the one behind each committed profile.
RETIRED = {"tools/ab.sh", "tools/c5_breakdown.sh", "tools/gpu_c5_prof.sh", "tools/gpu_event_check.sh",
           "tools/gpu_mfma_ab.sh", "tools/gpu_r02c.sh", "tools/gpu_r02d.sh", "tools/gpu_r02g.sh",
           "tools/gpu_r02j.sh", "tools/gpu_trace_shapes.sh", "tools/prof_shape.sh", "tools/profile.sh",
           "tools/summarize_profile.py", "tools/gpu_"}
BUILT = {"oracle/_ref", "tools/mfma_fp4_layout_probe"}   # build outputs (git-ignored)


def exists(p):
    if p in RETIRED or p in BUILT:
        return True
    # profiles/README.md lists files relative to profiles/
    for base in (ROOT, os.path.join(ROOT, PKG), os.path.join(ROOT, "profiles")):
        full = os.path.join(base, p)
        if os.path.exists(full):
            return True
        if p[-1] in "_-":                              # a family: `csrc/benor_w_`*.hip
            d, stem = os.path.split(full)
            if os.path.isdir(d) and any(f.startswith(stem) for f in os.listdir(d)):
                return True
    return False


def test_retired_tools_are_gone_and_noted():
    for p in RETIRED:
        assert not os.path.exists(os.path.join(ROOT, p)), p
    notes = open(os.path.join(ROOT, "profiles", "README.md"), encoding="utf-8").read()
    assert "tools/gpu.sh" in notes and "replaced" in notes


@pytest.mark.parametrize("doc", DOCS)
def test_cited_paths_exist(doc):
    missing = [p for p in cited_paths(doc) if not exists(p)]
    assert not missing, f"{doc} cites paths that are not in the repo: {missing}"


def test_profile_index_entries_exist():
    """profiles/README.md names each session's files relative to profiles/."""
    text = open(os.path.join(ROOT, "profiles", "README.md"), encoding="utf-8").read()
    names = {m for m in re.findall(r"`(r0\d[^`\s]*)`", text) if not any(c in m for c in "*<>{}") and "-vN_" not in m}   # r01-vN_: a template
    assert len(names) > 50
    missing = sorted(n for n in names if not os.path.exists(os.path.join(ROOT, "profiles", n)))
    assert not missing, f"profiles/README.md indexes files that are not in profiles/: {missing}"


# ------------------------------------------------- boundary text vs code
def test_random_stop_schedule_limits_match_the_code():
    """A random /stop schedule (crash_count, crash_window) is planned at every
    N <= BO_MAX_N (bo_kernel_for: the event-level family), so neither the C ABI
    header nor INTEGRATION.md may state a lower network-size limit for it."""
    import benor

    for N, F in ((10, 4), (256, 85), (1024, 341), (4096, 1365)):
        k = benor.kernel_for(N, F, [i < F for i in range(N)], mode=benor.BO_MODE_EVENT, k_max=16,
                             crash_count=3, crash_window=1000)
        assert k == benor.BO_KERNEL_EVENT, (N, k)
    hdr = open(os.path.join(ROOT, "include", "benor.h"), encoding="utf-8").read()
    integ = open(os.path.join(ROOT, "INTEGRATION.md"), encoding="utf-8").read()
    for text, name in ((hdr, "benor.h"), (integ, "INTEGRATION.md")):
        for line in text.splitlines():
            if "crash_count" in line:
                assert not re.search(r"N\s*(<=|≤|<)\s*(\d+)", line) or re.search(r"N\s*(<=|≤)\s*4096", line), \
                    f"{name}: {line.strip()}"
    assert "needs N <= 256" not in hdr


# ------------------------------------------------- environment knobs
CSRC = os.path.join(ROOT, PKG, "csrc")


def _csrc_text():
    out = {}
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".h", ".cpp", ".c")):
            out[f] = open(os.path.join(CSRC, f), encoding="utf-8").read()
    return out


def test_one_getenv_and_every_knob_registered():
    """The library reads the environment in one place (benor::knob, over the
    kKnobs table); every knob a source names is registered there, mirrored by
    benor.KNOBS and documented in DESIGN.md; no dropped A/B knob survives."""
    import benor

    src = _csrc_text()
    getenv = [(f, n) for f, t in src.items() for n in re.findall(r"\bgetenv\s*\(", t)]
    assert [f for f, _ in getenv] == ["benor_runtime.cpp"], getenv
    rt = src["benor_runtime.cpp"]
    table = rt[rt.index("constexpr KnobSpec kKnobs[]"):]
    table = table[:table.index("};")]
    registered = dict(re.findall(r'\{"(BENOR_[A-Z0-9_]+)",\s*"(\w+)"\}', table))
    used = {n for t in src.values() for n in re.findall(r'knob(?:_u32|_is)?\("(BENOR_[A-Z0-9_]+)"', t)}
    assert used <= set(registered), used - set(registered)
    assert set(registered) <= used, set(registered) - used          # no registered knob left unused
    assert registered == benor.KNOBS
    design = open(os.path.join(ROOT, "DESIGN.md"), encoding="utf-8").read()
    for name in registered:
        assert f"`{name}`" in design, name
    for dropped in ("BENOR_RANDOM_V1", "BENOR_COOP_PF", "BENOR_COOP_EXP", "BENOR_COOP_CBIAS", "BENOR_COOP_NT",
                    "BENOR_CONT_FULL_GRID", "BENOR_SMALL_FORM", "BENOR_EVENT_FAST"):
        assert all(dropped not in t for t in src.values()), dropped
