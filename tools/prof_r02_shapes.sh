#!/bin/bash
# r02 per-shape profiles: kernel trace of the perf-matrix shapes, then PMC
# passes (tools/prof_shape.sh) for the lane kernel (N=10, F=4), the W kernel at
# configs[2] (N=256, F=85) and random delivery (N=1024, f=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof_r02_trace
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r02_trace" -o shapes -- \
  python3 "$R/tools/perf_matrix.py" --shapes "10,4,4,0,20000000;256,85,85,0,10000000;1024,341,0,1,100000;10,4,4,2,2000000" \
  > "$R/gpurun_out/prof_r02_trace/pm.jsonl" 2>&1 ) || exit $?
for spec in "lane10:10,4,4,0,20000000" "n256:256,85,85,0,10000000" "rd1024:1024,341,0,1,100000"; do
  TAG=r02-${spec%%:*} SHAPE=${spec#*:} bash tools/prof_shape.sh || exit $?
done
echo done
