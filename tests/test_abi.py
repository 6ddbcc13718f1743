"""C ABI boundary checks that need no GPU (CPU suite).

* libbenor.so loads and exports every entry point include/benor.h declares.
* The host-side half of the reference surface behaves like the reference
  without any device work: launch validation (launchNodes.ts:10-13), initial
  NodeState (node.ts:21-26), /status (node.ts:33-39), /stop (node.ts:191-194).
  These are the reference's "Project is setup correctly" tests
  (benorconsensus.test.ts:45-118), verbatim in intent.
* Compute entry points fail loudly without a device (no CPU fallback).
"""
import os
import re
import subprocess

import pytest

import benor
from conftest import ROOT, check_reference_expectations

HEADER = os.path.join(ROOT, "include", "benor.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(bo_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_python_mirror_symbols():
    assert sorted(benor.EXPORTED_SYMBOLS) == header_symbols()


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", benor.LIB_PATH], check=True, capture_output=True,
                         text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing
    L = benor.lib()
    for s in header_symbols():
        assert hasattr(L, s)
    assert L.bo_abi_version() == 8
    assert L.bo_hist_len(64) == 65 * 3 + 1


def test_library_targets_gfx950():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          f"--input={benor.LIB_PATH}"], capture_output=True, text=True)
    # the offload bundle lives in .hip_fatbin; fall back to scanning the file
    data = open(benor.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_launch_errors(reference_cases):
    for e in reference_cases["launch_errors"]:
        with pytest.raises(benor.Error, match=re.escape(e["error"])):
            benor.launchNetwork(e["N"], e["F"], e["init"], e["faulty"])


def test_setup_cases_status(reference_cases):
    for case in reference_cases["cases"]:
        if case["start"]:
            continue
        N = case["N"]
        servers = benor.launchNetwork(N, sum(case["faulty"]), case["init"], case["faulty"])
        assert len(servers) == N
        statuses = [benor.getStatus(i) for i in range(N)]
        check_reference_expectations(case, benor.getNodesState(N), statuses)
        benor.stopConsensus(N)
        assert all(benor.getStatus(i) == (500, "faulty") for i in range(N))   # node.ts:191-194, :33-35
        for s in servers:
            s.close(lambda: s.closeAllConnections())


def test_initial_state_before_start():
    fl = [True, False, False, False, False]
    benor.launchNetwork(5, 1, [1, 0, "?", 1, 0], fl)
    st = benor.getNodesState(5)
    assert st[0] == {"killed": True, "x": None, "decided": None, "k": None}
    assert st[2] == {"killed": False, "x": "?", "decided": False, "k": 0}
    assert not benor.reachedFinality(st)


def test_state_records_decode_as_single_reads():
    """getNodesState decodes each distinct bo_node_state record once
    (benor._state_dicts); every dict equals the per-record decoding and is a
    separate object."""
    recs = [(0, 1, 1, 0, 3), (1, -1, -1, 0, -1), (0, 2, 0, 0, 7), (1, 0, 1, 0, 12), (0, 1, 1, 0, 3)]
    arr = (benor.NodeStateC * len(recs))()
    for r, (kl, x, d, pad, k) in zip(arr, recs):
        r.killed, r.x, r.decided, r.pad, r.k = kl, x, d, pad, k
    got = benor._state_dicts(arr, len(recs))
    assert got == [benor._state_dict(arr[i]) for i in range(len(recs))]
    assert got[0] is not got[4]
    got[0]["k"] = 99
    assert got[4]["k"] == 3


def test_reference_accepts_what_it_accepts():
    # F > N/2, '?' initial values, F == N are all accepted (launchNodes.ts:10-13
    # is the only validation; start.ts:25-29 rejects F > N/2 only in the demo).
    benor.launchNetwork(4, 3, ["?", 1, 0, 1], [True, True, True, False])
    benor.launchNetwork(2, 2, [1, 1], [True, True])
    assert benor.getNodesState(2)[0]["x"] is None


def test_second_start_without_gpu_work():
    """A start that stalls (a node stopped first: fewer than N-F senders,
    node.ts:52) needs no device; a second start is refused either way --
    the reference's inboxes persist across /start (node.ts:29-30)."""
    nodes = benor.launchNetwork(5, 1, [1, 1, 1, 0, 0], [False, False, False, False, True])
    nodes[0]._net.stop_node(0)
    benor.startConsensus(5, seed=3)
    assert [s["k"] for s in benor.getNodesState(5)] == [0, 1, 1, 1, None]
    benor.startConsensus(5, seed=3)                     # resolves, runs nothing (the reference answers 200)
    assert [s["k"] for s in benor.getNodesState(5)] == [0, 1, 1, 1, None]
    with pytest.raises(RuntimeError, match="libbenor error 8: consensus already started"):
        benor.startConsensus(5, seed=3, strict=True)


def test_network_create_null_arrays():
    L = benor.lib()
    import ctypes

    h = ctypes.c_void_p()
    assert L.bo_network_create(3, 0, None, 3, None, 3, ctypes.byref(h)) == benor.BO_ERR_INVALID_ARGUMENT
    assert L.bo_network_create(0, 0, None, 0, None, 0, ctypes.byref(h)) == benor.BO_OK
    L.bo_network_destroy(h)


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present: the loud-failure path is not reachable")
def test_no_silent_cpu_fallback():
    benor.launchNetwork(5, 0, [1] * 5, [False] * 5)
    with pytest.raises(RuntimeError, match="libbenor error 4"):
        benor.startConsensus(5, seed=1)
    with pytest.raises(RuntimeError, match="libbenor error 4"):
        benor.TrialsPlan(10, 4)


def test_library_built_from_these_sources():
    """libbenor.so bakes the digest of the kernel sources it was built from
    (Makefile KSHA); build() rebuilds on a mismatch and smoke() refuses one."""
    import sys

    sys.path.insert(0, ROOT)
    import __graft_entry__ as g

    assert benor.kernel_version() == g.kernel_digest()


def test_digest_covers_runtime_and_abi_header():
    """A change to the runtime (plans, dispatch, grid and deferral sizing) or
    to the C ABI header alone changes the digest, so the check above fails
    on a library built before it."""
    import sys

    sys.path.insert(0, ROOT)
    import __graft_entry__ as g

    srcs = g.digest_sources()
    rt = os.path.join(g.PKG, "csrc", "benor_runtime.cpp")
    hdr = os.path.join(ROOT, "include", "benor.h")
    assert rt in srcs and hdr in srcs
    base = g.kernel_digest()
    for f in (rt, hdr):
        assert g.kernel_digest({f: open(f, "rb").read() + b"\n// edit\n"}) != base
