#!/bin/bash
# r02 (session 3): matrix-core GPU tests, counter list, A/B of the SURE
# P-phase tail change over the matrix-core shapes, and a short bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mfma.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_mfma.log 2>&1
rc=$?; tail -3 gpurun_out/t_mfma.log; echo tests_rc=$rc
[ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 60 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1); echo list_rc=$?
AB_LIBS="base new" AB_SHAPES="256,85,85,0,200000000;1024,341,341,0,100000000;512,170,170,0,100000000;1024,0,0,0,20000000" bash tools/ab.sh || exit 1
cat gpurun_out/ab.jsonl
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_q.log 2>&1; echo bench_rc=$?
