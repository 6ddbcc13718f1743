#!/bin/bash
# One parameterised GPU-box session (replaces round 2's per-session gpu_*.sh
# wrappers).  Usage, as a gpurun command:
#
#   TAG=r03-v1 bash tools/gpu.sh smoke tests bench trace pmc:lane10 pmc:n256 ab c5 matrix
#
# Steps run in the order given, each under its own time limit, and the
# session stops at the first step that fails (no GPU step runs after a fault,
# abort or time limit).  Output goes to gpurun_out/<TAG>/; profiles/README.md
# says which files were copied into profiles/ from which step.
#
#   smoke           __graft_entry__.smoke()
#   tests           pytest -m gpu (PYTEST_ARGS: test paths / options, default the whole GPU suite;
#                   PYTEST_K: a -k expression, spaces allowed)
#   probe           tools/mfma_fp4_layout_probe (e2m1 MFMA K pairing)
#   bench           python bench.py (BENCH_ARGS, default the driver's --steps 20 --warmup 5)
#   trace           rocprofv3 --kernel-trace --stats of the same bench command
#   pmc:<shape>     PMC passes (PMC_GROUPS, '|'-separated, one rocprofv3 run each) over one
#                   tools/perf_matrix.py shape; <shape> is a key of SHAPES below or N,F,f,mode,trials
#   ab              tools/perf_matrix.py over AB_SHAPES for each build in AB_LIBS
#                   ("new" = the in-tree library, X = ab/libbenor_X.so), twice, alternating
#   abenv           as ab, one library, variants chosen by environment: AB_ENVS is a
#                   space-separated list of name=VAR:value,VAR:value ("new=" = no variables)
#   abin            tools/ab_inproc.py: AB_VARIANTS over AB_SHAPES ("N,F,trials;..."), interleaved
#                   rounds in one process (median / min per variant)
#   burstenv        as burst, once per AB_ENVS variant, twice, alternating
#   burst           tools/burst_time.py over BURST_SHAPES (10 back-to-back launches per shape)
#   c5              the C5 sweep (CSV compared with results/$C5_REF) and its per-N breakdown
#   c5phases        tools/c5_phases.py: the C5 sweep's wall time split (plans / queue / drain / read-back), twice
#   c5trace         the same under rocprofv3 --kernel-trace --stats
#   matrix          tools/perf_matrix.py over its built-in shape list
#   liveprof        tools/live_profile.py (LIVEPROF_ARGS): a live run's batch counters and cycle split
#   livepmc         PMC passes (PMC_GROUPS) over tools/live_profile.py (LIVEPROF_ARGS)
#   jslat           tools/js_latency.js (JSLAT_REPS): the same through the N-API addon (the JS drop-in)
#   netlat          tools/net_latency.py (NETLAT_ARGS): the reference's launch + start + final states
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
TAG=${TAG:-scratch}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp

declare -A SHAPES=(
  [lane10]="10,4,4,0,1000000"          # BASELINE configs[1] at its own trial count (lane kernel)
  [lane10l]="10,4,4,0,20000000"        # the same, steady state
  [lane105]="10,5,5,0,1000000"         # configs[1]'s F > N/2 no-decision case
  [n256]="256,85,85,0,10000000"        # configs[2] (small matrix-core kernel)
  [n256l]="256,85,85,0,200000000"
  [bench]="1024,341,341,0,100000000"   # configs[3] (the headline)
  [big1365]="4096,1365,1365,0,1000000" # big-network matrix-core kernel
  [big0]="4096,0,0,0,400000"
  [rd1024]="1024,341,0,1,200000"       # random delivery
  [ev256]="256,85,85,2,20000"          # event level
)
PMC_GROUPS=${PMC_GROUPS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT|SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA|SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE|FETCH_SIZE|WRITE_SIZE"}
BENCH_ARGS=${BENCH_ARGS:---steps 20 --warmup 5}

chk() {  # rc name
  echo "== $2 rc=$1"
  if [ "$1" -ne 0 ]; then echo "stopping after $2"; exit "$1"; fi
}

for step in "$@"; do
  case $step in
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      chk $? smoke; tail -1 "$OUT/smoke.log";;
    tests)
      timeout -k 10 ${TESTS_TIMEOUT:-900} python -u -m pytest ${PYTEST_ARGS:-tests} ${PYTEST_K:+-k "$PYTEST_K"} -m gpu ${PYTEST_X--x} -v --durations=30 --timeout 200 --timeout-method thread \
        > "$OUT/tests.log" 2>&1
      rc=$?; tail -3 "$OUT/tests.log"; chk $rc tests;;
    probe)
      timeout -k 10 60 "$R/tools/mfma_fp4_layout_probe" > "$OUT/fp4_probe.txt" 2>&1
      rc=$?; tail -3 "$OUT/fp4_probe.txt"; chk $rc probe;;
    bench)
      timeout -k 10 400 python -u bench.py $BENCH_ARGS > "$OUT/bench.log" 2>&1
      rc=$?; tail -c 600 "$OUT/bench.log"; echo; chk $rc bench;;
    trace)
      (cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
        python3 "$R/bench.py" $BENCH_ARGS > "$OUT/trace_bench.log" 2>&1)
      chk $? trace;;
    pmc:*)
      key=${step#pmc:}; shape=${SHAPES[$key]:-$key}; tag=$(echo "$key" | tr ',' '_')
      i=0; mkdir -p "$OUT/pmc_$tag"
      IFS='|' read -r -a GRPS <<< "$PMC_GROUPS"
      for grp in "${GRPS[@]}"; do
        i=$((i+1))
        (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_$tag/p$i" -o pmc -- \
          python3 "$R/tools/perf_matrix.py" --shapes "$shape" > "$OUT/pmc_$tag/p$i.log" 2>&1)
        chk $? "pmc $key pass $i ($grp)"
      done;;
    livepmc)
      i=0; mkdir -p "$OUT/livepmc"
      IFS='|' read -r -a GRPS <<< "$PMC_GROUPS"
      for grp in "${GRPS[@]}"; do
        i=$((i+1))
        (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/livepmc/p$i" -o pmc -- \
          python3 "$R/tools/live_profile.py" $LIVEPROF_ARGS > "$OUT/livepmc/p$i.log" 2>&1)
        chk $? "livepmc pass $i ($grp)"
      done;;
    ab)
      for rep in 1 2; do
        for lib in ${AB_LIBS:-base new}; do
          if [ "$lib" = new ]; then unset BENOR_LIB_PATH; else export BENOR_LIB_PATH="$R/ab/libbenor_$lib.so"; fi
          timeout -k 10 300 python -u tools/perf_matrix.py --shapes "${AB_SHAPES:?AB_SHAPES}" 2>/dev/null \
            | sed "s/^{/{\"lib\": \"$lib\", /" >> "$OUT/ab.jsonl"
          chk $? "ab $lib"
        done
      done
      unset BENOR_LIB_PATH;;
    abenv)
      for rep in 1 2; do
        for spec in ${AB_ENVS:?AB_ENVS}; do
          name=${spec%%=*}; vars=${spec#*=}
          envs=(); IFS=',' read -r -a kv <<< "$vars"
          for x in "${kv[@]}"; do [ -n "$x" ] && envs+=("${x%%:*}=${x#*:}"); done
          env "${envs[@]}" timeout -k 10 300 python -u tools/perf_matrix.py --shapes "${AB_SHAPES:?AB_SHAPES}" 2>/dev/null \
            | sed "s/^{/{\"lib\": \"$name\", /" >> "$OUT/ab.jsonl"
          chk $? "abenv $name"
        done
      done;;
    abin)
      timeout -k 10 600 python -u tools/ab_inproc.py --variants "${AB_VARIANTS:?AB_VARIANTS}" --shapes "${AB_SHAPES:?AB_SHAPES}" \
        ${AB_ARGS:-} > "$OUT/ab_inproc.jsonl" 2> "$OUT/ab_inproc.err"
      chk $? abin; cat "$OUT/ab_inproc.jsonl";;
    burstenv)
      for rep in 1 2; do
        for spec in ${AB_ENVS:?AB_ENVS}; do
          name=${spec%%=*}; vars=${spec#*=}
          envs=(); IFS=',' read -r -a kv <<< "$vars"
          for x in "${kv[@]}"; do [ -n "$x" ] && envs+=("${x%%:*}=${x#*:}"); done
          env "${envs[@]}" timeout -k 10 300 python -u tools/burst_time.py "${BURST_SHAPES:?BURST_SHAPES}" 2>/dev/null \
            | sed "s/^{/{\"lib\": \"$name\", /" >> "$OUT/burst.jsonl"
          chk $? "burstenv $name"
        done
      done;;
    burst)
      timeout -k 10 300 python -u tools/burst_time.py "${BURST_SHAPES:?BURST_SHAPES}" >> "$OUT/burst.jsonl"
      chk $? burst; cat "$OUT/burst.jsonl";;
    c5)
      C5=$OUT/c5; mkdir -p "$C5"
      (cd ben-or-consensus-algorithm_amd && timeout -k 10 150 python -u -m benor.cli sweep --out "$C5/sweep.csv" 2> "$C5/full.json")
      chk $? c5
      if cmp -s "$C5/sweep.csv" "results/${C5_REF:-r02_sweep_c5.csv}"; then echo "csv identical" | tee "$C5/cmp.txt"
      else echo "csv differs" | tee "$C5/cmp.txt"; fi
      cat "$C5/full.json"
      for N in 64 128 256 512 1024 2048 4096; do
        (cd ben-or-consensus-algorithm_amd && timeout -k 10 120 python -u -m benor.cli sweep --N $N --trials 153391680 \
          --out "$C5/n$N.csv" 2> "$C5/n$N.json")
        chk $? "c5 N=$N"
      done;;
    c5phases)
      timeout -k 10 200 python -u tools/c5_phases.py ${C5P_ARGS:-} > "$OUT/c5_phases.jsonl" 2> "$OUT/c5_phases.err"
      chk $? c5phases; cat "$OUT/c5_phases.jsonl";;
    c5trace)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5trace" -o c5 -- \
        python3 "$R/tools/c5_phases.py" > "$OUT/c5trace.log" 2>&1)
      chk $? c5trace;;
    matrix)
      timeout -k 10 400 python -u tools/perf_matrix.py > "$OUT/perf_matrix.jsonl" 2>&1
      chk $? matrix;;
    liveprof)
      timeout -k 10 300 python -u tools/live_profile.py ${LIVEPROF_ARGS:-} > "$OUT/live_profile.jsonl" 2> "$OUT/live_profile.err"
      chk $? liveprof; cat "$OUT/live_profile.jsonl";;
    netlat)
      timeout -k 10 400 python -u tools/net_latency.py ${NETLAT_ARGS:---reps 60} > "$OUT/net_latency.jsonl" 2> "$OUT/net_latency.err"
      chk $? netlat; cat "$OUT/net_latency.jsonl";;
    jslat)
      timeout -k 10 300 node tools/js_latency.js ${JSLAT_REPS:-60} > "$OUT/js_latency.jsonl" 2> "$OUT/js_latency.err"
      chk $? jslat; cat "$OUT/js_latency.jsonl";;
    *)
      echo "unknown step $step"; exit 2;;
  esac
done
echo "== done"
