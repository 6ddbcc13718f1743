set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -5 gpurun_out/tests.log; echo tests_rc=$rc
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u tools/perf_matrix.py --shapes "10,4,2,1,2000000;100,30,10,1,200000;1024,341,300,1,200000;1024,341,0,1,100000;4096,1365,0,1,10000;256,85,0,1,1000000;10,4,4,0,20000000" > gpurun_out/pm.jsonl 2>gpurun_out/pm.err; echo pm_rc=$?
