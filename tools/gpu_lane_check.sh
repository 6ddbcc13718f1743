set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -5 gpurun_out/tests.log; echo tests_rc=$rc
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u tools/perf_matrix.py --shapes "5,1,1,0,20000000;10,4,4,0,20000000;12,6,6,0,2000000;64,0,0,0,10000000;10,5,5,0,2000000;48,20,20,0,10000000" > gpurun_out/pm.jsonl 2>gpurun_out/pm.err; echo pm_rc=$?
