#!/bin/bash
# GPU session helper: runs smoke -> gpu tests -> bench, each under its own time
# limit; stops at the first crash/abort/timeout (exit > 1), continues past
# plain test failures (exit 1) so the bench still reports.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in ${STEPS:-smoke tests bench}; do
  case $s in
    smoke) step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()";;
    tests) step tests 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread;;
    bench) step bench 300 python -u bench.py ${BENCH_ARGS:---steps 5 --warmup 1 --cpu-seconds 10};;
  esac
done
