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
