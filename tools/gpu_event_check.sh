#!/bin/bash
# Event-mode GPU session: parity tests (-k event), then event-mode throughput.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "event" --timeout 300 --timeout-method thread > gpurun_out/tests_event.log 2>&1
rc=$?; tail -4 gpurun_out/tests_event.log; echo tests_rc=$rc
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/perf_matrix.py --shapes "${SHAPES:-10,4,4,2,2000000;32,10,10,2,200000;64,21,21,2,100000;128,42,42,2,20000;256,85,85,2,2000}" > gpurun_out/pm_event.jsonl 2> gpurun_out/pm_event.err
echo pm_rc=$?
