set -e
TAG=r03-v5 PYTEST_ARGS="tests/test_mfma_small.py" bash tools/gpu.sh tests
for b in 0 1 2 4 8; do
  if [ $b = 0 ]; then unset BENOR_BLOCKS_PER_CU; else export BENOR_BLOCKS_PER_CU=$b; fi
  TAG=r03-v5 BURST_SHAPES="10,4,1000;10,4,1000000;10,4,20000000;5,1,1000000" bash tools/gpu.sh burst > /dev/null
  echo "bpc=$b"; tail -4 gpurun_out/r03-v5/burst.jsonl
done
