#!/bin/bash
# Matrix-core PMC of the big-network kernel on a few shapes (one pass each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for s in ${PMC_SHAPES:-"4096,0,0,0,1000000" "4096,1365,1365,0,1000000" "2048,682,682,0,2000000"}; do
  tag=$(echo $s | cut -d, -f1-2 | tr , _)
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_big_$tag -o pmc -- python3 $R/tools/perf_matrix.py --shapes "$s" > $R/gpurun_out/pmc_big_$tag.log 2>&1 || { echo pmc_fail $tag; exit 1; }
done
echo pmc_ok
