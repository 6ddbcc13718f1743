set -e
T=r03-v11
mkdir -p gpurun_out/$T
TAG=$T PYTEST_ARGS="tests/test_mfma_small.py" bash tools/gpu.sh tests
for v in packed lane; do
  if [ $v = lane ]; then export BENOR_NO_MFMA=1; else export BENOR_SMALL_MIN_TRIALS=0; fi
  TAG=$T BURST_SHAPES="5,1,20000000;5,1,40000000;12,4,20000000;20,4,20000000;40,8,20000000;10,4,40000000" bash tools/gpu.sh burst > /dev/null
  unset BENOR_NO_MFMA BENOR_SMALL_MIN_TRIALS
done
cat gpurun_out/$T/burst.jsonl
TAG=$T bash tools/gpu.sh bench trace pmc:bench pmc:lane10 pmc:lane10l
