set -e
T=r03-v10
mkdir -p gpurun_out/$T
TAG=$T PYTEST_ARGS="tests/test_mfma_small.py" bash tools/gpu.sh tests
for v in packed lane; do
  if [ $v = lane ]; then export BENOR_NO_MFMA=1; else export BENOR_SMALL_MIN_TRIALS=0; fi
  TAG=$T BURST_SHAPES="10,4,1000000;10,4,2000000;10,4,4000000;10,4,8000000;10,4,20000000;5,1,1000000;5,1,8000000" bash tools/gpu.sh burst > /dev/null
  echo "$v"; tail -7 gpurun_out/$T/burst.jsonl
  unset BENOR_NO_MFMA BENOR_SMALL_MIN_TRIALS
done
BENOR_SMALL_MIN_TRIALS=0 TAG=r03-v10 bash tools/gpu.sh pmc:lane10 pmc:lane10l pmc:n256 pmc:n256l
BENOR_NO_MFMA=1 TAG=r03-v10-lane bash tools/gpu.sh pmc:lane10 pmc:lane10l
