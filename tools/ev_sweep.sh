#!/bin/bash
# Event-mode occupancy sweep: lanes per CU (BENOR_EVENT_LANES_PER_CU) x N -> gpurun_out/ev.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for pc in ${PCS:-128 256 384 512 768}; do
  BENOR_EVENT_LANES_PER_CU=$pc timeout -k 10 200 python -u tools/perf_matrix.py --shapes "${EV_SHAPES:-5,1,1,2,8000000;10,4,4,2,4000000;20,6,6,2,1000000;32,10,10,2,400000;64,21,21,2,200000}" | sed "s/^{/{\"per_cu\": $pc, /" >> gpurun_out/ev.jsonl || exit 1
done
