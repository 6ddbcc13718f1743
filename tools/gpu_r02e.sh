#!/bin/bash
# r02 (session 3): lane kernel with sign-bit tallies -- full GPU suite, then
# an A/B against the previous build over the lane-kernel shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -2 gpurun_out/tests.log; echo tests_rc=$rc; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/ab.jsonl
AB_LIBS="base new" AB_SHAPES="5,1,1,0,20000000;10,4,4,0,20000000;10,4,4,0,1000000;10,5,5,0,20000000;3,1,1,0,20000000;20,6,6,0,20000000;40,8,8,0,10000000;48,20,20,0,10000000;64,21,21,0,10000000;33,0,0,0,10000000" bash tools/ab.sh || exit 1
