#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof summary. Each GPU step has its
# own time limit; a crash/abort/timeout (rc >= 124 or signal) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-run}
mkdir -p "$OUT"
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fatal rc=$rc in $name: stopping"; exit $rc
  fi
  return 0
}
for s in ${STEPS:-pytest smoke bench prof}; do
  case $s in
    pytest) step pytest_gpu 1500 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 900 python bench.py ${BENCH_ARGS:-} ;;
    prof)   step prof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
  esac
done
echo "all steps done"
