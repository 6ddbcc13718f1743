#!/bin/bash
# A/B of libbenor builds over lockstep shapes (perf_matrix), alternating runs
# on one box: gpurun_out/ab.jsonl.  AB_LIBS names the builds (default
# "base new"): "new" = the in-tree build, any other name X = ab/libbenor_X.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SH=${AB_SHAPES:-"64,21,21,0,20000000;128,42,42,0,20000000;256,85,85,0,20000000;512,170,170,0,10000000;1024,341,341,0,20000000;1024,0,0,0,4000000;2048,682,682,0,1000000"}
for rep in 1 2; do
  for lib in ${AB_LIBS:-base new}; do
    if [ $lib = new ]; then unset BENOR_LIB_PATH; else export BENOR_LIB_PATH=$PWD/ab/libbenor_$lib.so; fi
    timeout -k 10 200 python -u tools/perf_matrix.py --shapes "$SH" 2>/dev/null | sed "s/^{/{\"lib\": \"$lib\", /" >> gpurun_out/ab.jsonl || exit 1
  done
done
