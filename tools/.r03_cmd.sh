set -e
T=r03-v8
mkdir -p gpurun_out/$T
for t in 1000000 20000000; do for b in 1 2 4; do for c in 0 1 2 8; do timeout -k 10 60 tools/small_phase_probe $t $b $c; done; done; done > gpurun_out/$T/phases.txt 2>&1
TAG=$T PYTEST_ARGS="tests/test_mfma_small.py" bash tools/gpu.sh tests
for c in 0 1 2 4; do for b in 0 4; do
  if [ $b = 0 ]; then unset BENOR_BLOCKS_PER_CU; else export BENOR_BLOCKS_PER_CU=$b; fi
  export BENOR_SMALL_CHUNK=$c
  TAG=$T BURST_SHAPES="10,4,1000000;10,4,20000000;5,1,1000000" bash tools/gpu.sh burst > /dev/null
  echo "chunk=$c bpc=$b"; tail -3 gpurun_out/$T/burst.jsonl
done; done
