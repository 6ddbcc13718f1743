#!/bin/bash
# Round-2 GPU session: the new blocked-kernel parity cases, then the bench
# profile (tools/profile.sh) under TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "blocked_kernel_block_sizes" --timeout 200 --timeout-method thread > gpurun_out/tests_blocked.log 2>&1
rc=$?; tail -3 gpurun_out/tests_blocked.log; echo tests_rc=$rc
[ $rc -gt 1 ] && exit $rc
TAG=${TAG:-r02} bash tools/profile.sh
