#!/bin/bash
# r02 (session 3): short-launch grid sweep (lane kernel tail), and MFMA / VALU
# co-execution counters for the configs[2] matrix-core kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/lane_grid_sweep.py > gpurun_out/lane_grid.jsonl 2> gpurun_out/lane_grid.err; echo sweep_rc=$?
cat gpurun_out/lane_grid.jsonl
R=$PWD
cd /tmp && export TMPDIR=/tmp
for s in "256,85,85,0,20000000" "1024,341,341,0,20000000"; do
  tag=$(echo $s | cut -d, -f1)
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_mfma_$tag -o pmc -- python3 $R/tools/perf_matrix.py --shapes "$s" > $R/gpurun_out/pmc_mfma_$tag.log 2>&1 || { echo pmc_fail $tag; exit 1; }
done
echo pmc_ok
