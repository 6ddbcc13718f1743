#!/bin/bash
# Kernel-trace of short launches (tools/burst_time.py): kernel durations
# without the gaps between back-to-back launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/burst_trace -o burst -- python3 $R/tools/burst_time.py "${SHAPES:-10,4,1000000;10,4,100000;10,10,1000000}" > $R/gpurun_out/burst_trace.log 2>&1
echo rc=$?
