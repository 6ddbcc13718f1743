#!/bin/bash
# r02 (session 3): two trials per lane in the lane kernel -- full GPU suite,
# then burst timing of the lane shapes against the previous build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -2 gpurun_out/tests.log; echo tests_rc=$rc; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/burst_ab.jsonl
SH="10,4,1000000;5,1,1000000;10,5,1000000;20,6,1000000;10,4,20000000;5,1,20000000;10,5,20000000;20,6,20000000;31,10,10000000;64,21,10000000"
for rep in 1 2; do
  for lib in base new; do
    if [ $lib = new ]; then unset BENOR_LIB_PATH; else export BENOR_LIB_PATH=$PWD/ab/libbenor_$lib.so; fi
    timeout -k 10 200 python -u tools/burst_time.py "$SH" 2>/dev/null | sed "s/^{/{\"lib\": \"$lib\", /" >> gpurun_out/burst_ab.jsonl || exit 1
  done
done
