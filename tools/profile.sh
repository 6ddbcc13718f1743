#!/bin/bash
# Profiling session on the GPU box: VALU issue-rate probe, kernel-trace stats
# of the bench, PMC passes (each counter group in a pass of its own).
# Output under gpurun_out/prof_<tag>/ ; summaries are copied into profiles/ by hand.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r01}
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH_ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --cpu-seconds 0 --no-peak-probe --no-other-configs}
PMC_ARGS=${PMC_ARGS:---trials 100000000 --steps 1 --warmup 0 --cpu-seconds 0 --no-peak-probe --no-other-configs}
chk() { local rc=$1 name=$2; echo "== $name rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $name"; exit "$rc"; fi; }
if [ -z "$SKIP_PROBE" ]; then
  timeout -k 10 120 "$R/tools/valu_probe" > "$OUT/valu_probe.txt" 2>&1; chk $? probe
  cat "$OUT/valu_probe.txt"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
  python3 "$R/bench.py" $BENCH_ARGS > "$OUT/trace_bench.log" 2>&1; chk $? kernel-trace
tail -2 "$OUT/trace_bench.log"
i=0
# PMC_GROUPS: counter groups separated by '|', one rocprofv3 pass each
GROUPS_STR=${PMC_GROUPS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT|SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA|FETCH_SIZE|WRITE_SIZE"}
IFS='|' read -r -a GROUPS_ARR <<< "$GROUPS_STR"
for grp in "${GROUPS_ARR[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o pmc -- \
    python3 "$R/bench.py" $PMC_ARGS > "$OUT/pmc$i.log" 2>&1; chk $? "pmc$i ($grp)"
done
echo done
