#!/bin/bash
# rocprofv3 kernel-trace stats + PMC passes (one counter group per process) of
# the GF(16) EMS kernel over scripts/bench_ems.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-ems_prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--ebn0 2.0 --steps 2 --batch 16384 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o ems --output-format csv -- python3 scripts/bench_ems.py $ARGS > "$OUT/stats.log" 2>&1 || exit $?
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o pmc --output-format csv -- python3 scripts/bench_ems.py $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i rc=$?"; exit 1; }
done
echo done
