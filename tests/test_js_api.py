"""The reference's JS/TS surface (ben-or-consensus-algorithm_amd/js) driven by
tests/js/benorconsensus.test.js, a plain-Node re-expression of
__test__/tests/benorconsensus.test.ts.  The setup/validation cases need no
GPU; the finality cases run the kernel through the N-API addon."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SCRIPT = os.path.join(ROOT, "tests", "js", "benorconsensus.test.js")
ADDON = os.path.join(ROOT, "ben-or-consensus-algorithm_amd", "js", "benor.node")

needs_node = pytest.mark.skipif(shutil.which("node") is None or not os.path.exists(ADDON),
                                reason="node or the N-API addon is not available")


def _run(which):
    p = subprocess.run(["node", SCRIPT, which], capture_output=True, text=True, timeout=120)
    print(p.stdout, p.stderr)
    assert p.returncode == 0, p.stdout + p.stderr


@needs_node
def test_js_setup_cases():
    _run("setup")


@needs_node
@pytest.mark.gpu
def test_js_reference_suite():
    _run("all")


@needs_node
def test_js_typed_paths_agree_with_the_addon():
    """js/index.js encodes launchNetwork's arrays itself and decodes raw state
    records; the same errors and NodeState objects as the addon's per-element
    paths (tests/js/typed_paths.test.js, pre-run states: no GPU)."""
    p = subprocess.run(["node", os.path.join(ROOT, "tests", "js", "typed_paths.test.js")], capture_output=True,
                       text=True, timeout=120)
    print(p.stdout, p.stderr)
    assert p.returncode == 0, p.stdout + p.stderr


HTTP_SCRIPT = os.path.join(ROOT, "tests", "js", "http_facade.test.js")


def _run_http(which):
    p = subprocess.run(["node", HTTP_SCRIPT, which], capture_output=True, text=True, timeout=120)
    print(p.stdout, p.stderr)
    assert p.returncode == 0, p.stdout + p.stderr


@needs_node
def test_http_facade_setup_cases():
    """/status, /getState, /stop served on 3100+i."""
    _run_http("setup")


@needs_node
@pytest.mark.gpu
def test_http_facade_reference_suite():
    _run_http("all")


START_JS = os.path.join(ROOT, "ben-or-consensus-algorithm_amd", "js", "start.js")


@needs_node
def test_js_start_rejects_like_start_ts():
    """js/start.js re-states src/start.ts:22-29: its checks run before any GPU work."""
    p = subprocess.run(["node", START_JS, "--init", "1,1,1,1", "--faulty", "0,1,2"], capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == 1 and "Too many faulty nodes" in p.stderr
    p = subprocess.run(["node", START_JS, "--N", "5", "--init", "1,1,1,1", "--faulty", "0"], capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == 1 and "Lengths don't match" in p.stderr


@needs_node
@pytest.mark.gpu
def test_js_start_scenario():
    """`yarn start` (src/start.ts): N=10, nodes 0-3 faulty, all 1 -> live nodes decide 1."""
    p = subprocess.run(["node", START_JS, "--seed", "7"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    lines = p.stdout.strip().splitlines()
    assert len(lines) == 10
    assert all('"killed":true' in l for l in lines[:4])
    assert all('"decided":true' in l and '"x":1' in l for l in lines[4:])


def test_cli_int_parser():
    from benor.cli import _ints

    assert _ints("64, 128,2**10") == [64, 128, 1024]
    with pytest.raises(ValueError):
        _ints("__import__('os')")
