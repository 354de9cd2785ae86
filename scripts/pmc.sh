#!/bin/bash
# PMC passes over a short bench run (one counter group per process, as the
# MI355X guide prescribes: never combine --pmc with trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps ${PMC_STEPS:-2} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
if [ "${LIST:-0}" = 1 ]; then timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1; fi
i=0
for set in "${@}"; do
  i=$((i+1))
  echo "=== pass $i: $set"
  timeout -k 10 600 rocprofv3 --pmc $set -d "$OUT/p$i" -o pmc --output-format csv -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -2 "$OUT/p$i.log"
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
done
