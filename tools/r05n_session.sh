set -o pipefail
O=gpurun_out/r05-n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_live_stop.py tests/test_stop_schedule.py tests/test_js_api.py tests/test_gpu_parity.py -k "live or stop or event or js" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/net_latency.py --reps 100 > $O/net_latency_new.jsonl || exit 1
BENOR_LIB_PATH=$PWD/ab/libbenor_base.so timeout -k 10 300 python -u tools/net_latency.py --reps 100 > $O/net_latency_base.jsonl || exit 1
paste -d'\n' $O/net_latency_base.jsonl $O/net_latency_new.jsonl
