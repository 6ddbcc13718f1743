#!/bin/bash
# Matrix-core kernel session: its GPU tests (oracle parity, deferral), then an
# A/B of library builds (tools/ab.sh) over the matrix-core shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mfma.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_mfma.log 2>&1
rc=$?; tail -3 gpurun_out/t_mfma.log; echo tests_rc=$rc
[ $rc -ne 0 ] && exit $rc
AB_LIBS=${AB_LIBS:-"base new"} AB_SHAPES=${AB_SHAPES:-"256,85,85,0,200000000;1024,341,341,0,100000000;1024,0,0,0,20000000;256,0,0,0,50000000;1024,400,400,0,20000000;1000,300,300,0,20000000"} bash tools/ab.sh
rc=$?; cat gpurun_out/ab.jsonl; exit $rc
