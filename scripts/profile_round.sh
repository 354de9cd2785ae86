#!/bin/bash
# Kernel-trace stats + HBM PMC passes (FETCH_SIZE and WRITE_SIZE in separate
# runs) of the default bench workload; summaries go to gpurun_out/$RUN_TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-prof}
mkdir -p "$OUT"
ARGS="--steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-}"
run() { local name=$1; shift; echo "=== $name"; timeout -k 10 300 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run stats rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 bench.py $ARGS
run fetch rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o pmc --output-format csv -- python3 bench.py $ARGS
run write rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o pmc --output-format csv -- python3 bench.py $ARGS
run sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d "$OUT/sq" -o pmc --output-format csv -- python3 bench.py $ARGS
run sq2 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d "$OUT/sq2" -o pmc --output-format csv -- python3 bench.py $ARGS
echo done
