#!/bin/bash
# C5 sweep on one GPU: the full 224-cell run (CSV compared with the committed
# result) and the same per-cell budget per N, timed separately.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}/ben-or-consensus-algorithm_amd"
OUT=../gpurun_out/c5
mkdir -p $OUT
timeout -k 10 120 python -u -m benor.cli sweep --out $OUT/sweep.csv 2> $OUT/full.json || exit 1
cmp $OUT/sweep.csv ../results/${C5_REF:-r02_sweep_c5.csv} && echo "csv identical" > $OUT/cmp.txt || echo "csv differs" > $OUT/cmp.txt
for N in 64 128 256 512 1024 2048 4096; do
  timeout -k 10 120 python -u -m benor.cli sweep --N $N --trials 153391680 --out $OUT/n$N.csv 2> $OUT/n$N.json || exit 1
done
