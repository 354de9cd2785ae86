#!/bin/bash
# HBM bytes of the DVB-S2 flooding kernel: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-pmc_flood}
mkdir -p "$OUT"
DVB=$(python3 -c "import sys; sys.path.insert(0, 'tests'); from conftest import code_path; print(code_path('dvbs2_1_2.alist'))")
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/$c" -o pmc --output-format csv -- \
    python3 scripts/time_code.py "$DVB" --batch 2048 --T 50 --snr 1.0 --variant nms --reps 1 > "$OUT/$c.log" 2>&1 \
    || { echo "$c failed"; exit 1; }
  tail -1 "$OUT/$c.log"
done
