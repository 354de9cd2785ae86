#!/bin/bash
# A/B of scripts/time_code.py over values of one environment variable, interleaved rounds.
# usage: ab_code.sh VAR "v1 v2 ..." ROUNDS CODE [time_code args]   (CODE: a tests/golden/codes name)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VAR=$1; VALS=$2; ROUNDS=$3; CODE=$4; shift 4
ALIST=$(python3 -c "import sys; sys.path.insert(0, 'tests'); from conftest import code_path; print(code_path('$CODE'))")
mkdir -p gpurun_out/ab_code
for r in $(seq 1 $ROUNDS); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python3 scripts/time_code.py "$ALIST" "$@" > gpurun_out/ab_code/$VAR-$v-$r.log 2>&1 || { echo "fail $v"; tail -3 gpurun_out/ab_code/$VAR-$v-$r.log; exit 1; }
    echo "$VAR=$v $(tail -1 gpurun_out/ab_code/$VAR-$v-$r.log)"
  done
done
