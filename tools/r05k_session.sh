set -o pipefail
O=gpurun_out/r05-k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mfma_small.py tests/test_mfma.py tests/test_live_stop.py tests/test_stop_schedule.py tests/test_gpu_parity.py -k "mfma or live or stop or event" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/burst_time.py "10,4,1000000;10,4,20000000;5,1,1000000;16,7,3000000;10,4,1048577" > $O/burst.jsonl || exit 1
cat $O/burst.jsonl
timeout -k 10 120 python -u tools/timeline_report.py $O/tl.txt --run 10 4 1000000 > $O/timeline.md || exit 1
head -20 $O/timeline.md
timeout -k 10 300 python -u tools/net_latency.py --reps 100 > $O/net_latency_new.jsonl || exit 1
BENOR_LIB_PATH=$PWD/ab/libbenor_base.so timeout -k 10 300 python -u tools/net_latency.py --reps 100 > $O/net_latency_base.jsonl || exit 1
paste -d'\n' $O/net_latency_base.jsonl $O/net_latency_new.jsonl
TAG=r05-k AB_LIBS="base new" AB_SHAPES="256,85,85,0,10000000;256,85,85,0,40000000;1024,341,341,0,20000000;10,4,4,0,1000000;10,4,4,0,20000000" bash tools/gpu.sh ab || exit 1
cat $O/ab.jsonl
