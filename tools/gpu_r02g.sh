#!/bin/bash
# r02 (session 3): matrix-core continuation passes (rounds 2..3 of tied
# trials on the matrix cores) -- full GPU suite, then an A/B over KIND 1/2 shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -2 gpurun_out/tests.log; echo tests_rc=$rc; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/ab.jsonl
AB_LIBS="base new" AB_SHAPES="256,0,0,0,50000000;1024,0,0,0,20000000;1000,300,300,0,20000000;1024,400,400,0,20000000;512,170,170,0,50000000;128,0,0,0,50000000;256,85,85,0,100000000" bash tools/ab.sh || exit 1
