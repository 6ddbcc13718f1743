# burst A/B of two builds (ab/libbenor_base.so vs the in-tree library), alternating twice
# (TAG=... BURST_SHAPES="N,F,trials;..." bash tools/r05s_burst_ab.sh)
set -o pipefail
O=gpurun_out/${TAG:-r05-s}; mkdir -p $O
SH="${BURST_SHAPES:-10,4,1000000;5,1,1000000;10,4,4000000;10,4,20000000;16,7,3000000;32,0,2000000}"
for rep in 1 2; do
  BENOR_LIB_PATH=$PWD/ab/libbenor_base.so timeout -k 10 120 python -u tools/burst_time.py "$SH" | sed 's/^{/{"lib": "base", /' >> $O/burst_ab.jsonl || exit 1
  timeout -k 10 120 python -u tools/burst_time.py "$SH" | sed 's/^{/{"lib": "new", /' >> $O/burst_ab.jsonl || exit 1
done
cat $O/burst_ab.jsonl
