set -e
T=r03-v12
mkdir -p gpurun_out/$T
TAG=$T PYTEST_ARGS="tests/test_mfma_small.py" bash tools/gpu.sh tests
for b in 0 2 4 8; do
  if [ $b = 0 ]; then unset BENOR_BLOCKS_PER_CU; else export BENOR_BLOCKS_PER_CU=$b; fi
  BENOR_SMALL_MIN_TRIALS=0 TAG=$T BURST_SHAPES="10,4,1000000;10,4,4000000;10,4,20000000;5,1,1000000;5,1,20000000;20,4,20000000" bash tools/gpu.sh burst > /dev/null
  echo "bpc=$b"; tail -6 gpurun_out/$T/burst.jsonl
done
