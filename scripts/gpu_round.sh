#!/bin/bash
# One GPU pass: pytest -m gpu, smoke, the default bench line, and rocprofv3
# kernel-trace stats of the same bench command. Each step under its own time
# limit; the first failure ends the pass. Output: gpurun_out/$RUN_TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-round}
mkdir -p "$OUT"
step() { local name=$1 lim=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 900 python -u -m pytest ${PYTEST_TARGETS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python bench.py ${BENCH_ARGS:-}
if [ "${SKIP_PROF:-0}" != 1 ]; then
  step stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-}
fi
echo "done $(date +%T)"
