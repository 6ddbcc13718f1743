#!/bin/bash
# Kernel-trace stats of tools/perf_matrix.py over SHAPES (one rocprofv3 run):
# gpurun_out/trace_<TAG>/ ; per-kernel durations for launches that chain
# several kernels (matrix-core round 1 + W-kernel deferred trials).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-shapes}
OUT="$R/gpurun_out/trace_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o t -- \
  python3 "$R/tools/perf_matrix.py" --shapes "$SHAPES" > "$OUT/perf.log" 2>&1
rc=$?; cat "$OUT/perf.log" | grep '^{'; cat "$OUT"/*kernel_stats.csv; exit $rc
