#!/bin/bash
# Random-delivery parity + throughput, then the C5 sweep breakdown.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "random_delivery or fuzz" --timeout 300 --timeout-method thread > gpurun_out/tests_rd.log 2>&1
rc=$?; tail -3 gpurun_out/tests_rd.log; echo tests_rc=$rc
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/perf_matrix.py --shapes "10,4,2,1,2000000;100,30,10,1,200000;1024,341,300,1,200000;1024,341,0,1,100000;4096,1365,1000,1,20000" > gpurun_out/pm_rd.jsonl 2> gpurun_out/pm_rd.err || exit $?
bash tools/c5_breakdown.sh
