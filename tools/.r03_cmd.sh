set -e
T=r03-v14
mkdir -p gpurun_out/$T
TAG=$T PYTEST_ARGS="tests/test_mfma.py tests/test_c5.py tests/test_mfma_small.py" bash tools/gpu.sh tests
TAG=$T AB_SHAPES="4096,1365,1365,0,400000;4096,0,0,0,100000;2048,682,682,0,1000000;1500,200,200,0,1000000;3000,1400,1400,0,400000;256,85,85,0,20000000;128,42,42,0,20000000;200,66,66,0,10000000;1024,341,341,0,20000000;10,4,4,0,1000000;10,4,4,0,20000000" bash tools/gpu.sh ab > /dev/null
python tools/ab_report.py gpurun_out/$T/ab.jsonl
TAG=$T bash tools/gpu.sh c5
