#!/bin/bash
# r02 (session 3): A/B of SURE-kernel variants (software pipelining, shared
# bias registers) and a short bench with the lane-kernel grid heuristic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl
AB_LIBS="new pipe share pipeshare" AB_SHAPES="256,85,85,0,200000000;1024,341,341,0,100000000;190,63,63,0,200000000;898,299,299,0,100000000" bash tools/ab.sh || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_q.log 2>&1; echo bench_rc=$?
