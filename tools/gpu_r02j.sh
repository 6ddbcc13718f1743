#!/bin/bash
# r02 (session 3): event-level mode with the inbox counters in LDS (N <= 16)
# -- the event GPU tests, then an A/B over event shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "event or Event" --timeout 300 --timeout-method thread > gpurun_out/t_event.log 2>&1
rc=$?; tail -2 gpurun_out/t_event.log; echo tests_rc=$rc; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/ab.jsonl
AB_LIBS="${AB_LIBS:-base new}" AB_SHAPES="${AB_SHAPES:-10,4,4,2,2000000;5,1,1,2,2000000;16,5,5,2,1000000;12,3,3,2,1000000;32,10,10,2,200000}" bash tools/ab.sh || exit 1
