#!/bin/bash
# PMC passes (one counter group per process) over scripts/time_code.py on one code.
# usage: pmc_code.sh CODE "time_code args" "counters pass 1" "counters pass 2" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-pmc_code}
mkdir -p "$OUT"
CODE=$1; ARGS=$2; shift 2
ALIST=$(python3 -c "import sys; sys.path.insert(0, 'tests'); from conftest import code_path; print(code_path('$CODE'))")
if [ "${LIST:-0}" = 1 ]; then timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1; fi
i=0
for set in "$@"; do
  i=$((i+1))
  echo "=== pass $i: $set"
  timeout -k 10 300 rocprofv3 --pmc $set -d "$OUT/p$i" -o pmc --output-format csv -- python3 scripts/time_code.py "$ALIST" $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -1 "$OUT/p$i.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
done
