#!/bin/bash
# A/B of two libbenor builds over lockstep shapes (perf_matrix), alternating
# runs on one box: gpurun_out/ab.jsonl.  BASE = ab/libbenor_base.so (saved
# copy of the previous build), NEW = the in-tree build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SH=${AB_SHAPES:-"64,21,21,0,20000000;128,42,42,0,20000000;256,85,85,0,20000000;512,170,170,0,10000000;1024,341,341,0,20000000;1024,0,0,0,4000000;2048,682,682,0,1000000"}
for rep in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then export BENOR_LIB_PATH=$PWD/ab/libbenor_base.so; else unset BENOR_LIB_PATH; fi
    timeout -k 10 200 python -u tools/perf_matrix.py --shapes "$SH" 2>/dev/null | sed "s/^{/{\"lib\": \"$lib\", /" >> gpurun_out/ab.jsonl || exit 1
  done
done
