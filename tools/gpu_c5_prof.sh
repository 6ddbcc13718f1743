#!/bin/bash
# C5 sweep: per-N breakdown (CSV compared with the committed result), then a
# kernel-trace of the full sweep (time per kernel family).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/c5_breakdown.sh || exit 1
cat gpurun_out/c5/cmp.txt gpurun_out/c5/full.json
R=$PWD
cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R/ben-or-consensus-algorithm_amd
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c5_trace -o c5 -- python3 -m benor.cli sweep --out /tmp/c5.csv > $R/gpurun_out/c5_trace.log 2>&1
echo trace_rc=$?
