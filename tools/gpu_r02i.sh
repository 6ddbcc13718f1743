#!/bin/bash
# r02 (session 3): big-network matrix-core kernel with zero-start
# accumulators (bias added after the chunk loop; 124-131 VGPRs, 3 waves/SIMD)
# -- matrix-core GPU tests, then an A/B over big shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mfma.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_mfma.log 2>&1
rc=$?; tail -2 gpurun_out/t_mfma.log; echo tests_rc=$rc; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/ab.jsonl
AB_LIBS="${AB_LIBS:-base new}" AB_SHAPES="4096,1365,1365,0,2000000;4096,0,0,0,1000000;2048,682,682,0,4000000;1500,200,200,0,4000000;3000,1400,1400,0,2000000;2048,0,0,0,2000000;4096,2000,2000,0,2000000;1100,366,366,0,10000000" bash tools/ab.sh || exit 1
