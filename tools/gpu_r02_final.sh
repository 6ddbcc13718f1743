#!/bin/bash
# Round-2 profile session on the current kernels: smoke, GPU tests, the bench,
# tools/profile.sh under TAG (kernel trace + PMC incl. matrix-core counters and
# HBM traffic), then the C5 sweep breakdown.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; echo smoke_rc=$rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -2 gpurun_out/tests.log; echo tests_rc=$rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo bench_rc=$rc; [ $rc -ne 0 ] && exit $rc
SKIP_PROBE=1 TAG=${TAG:-r02-v6} PMC_GROUPS="${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT|SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE|FETCH_SIZE|WRITE_SIZE}" bash tools/profile.sh || exit $?
cd "${GRAFT_REPO_ROOT:-.}" && bash tools/c5_breakdown.sh && cat gpurun_out/c5/cmp.txt gpurun_out/c5/full.json
