#!/bin/bash
# Config 3 (DVB-S2 N=64800 R1/2, NMS alpha=1.25, T=50) at the reference's precision:
# kernel-trace stats and PMC passes (one counter group per rocprofv3 pass) of the
# flooding and the layered fp64 kernels, 2,048 codewords per launch (one warm-up
# launch + REPS timed ones).  Summaries: scripts/summarize_config3.py.
# usage: RUN_TAG=r05_config3 bash scripts/pmc_config3.sh  -> gpurun_out/$RUN_TAG/{flooding,layered}/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-config3}
BATCH=${BATCH:-2048}
REPS=${REPS:-1}
PREC=${PREC:-f64}
mkdir -p "$OUT"
DVB=$(python3 -c "import sys; sys.path.insert(0, 'tests'); from conftest import code_path; print(code_path('dvbs2_1_2.alist'))")
for sched in ${SCHEDS:-flooding layered}; do
  D="$OUT/$sched"; mkdir -p "$D"
  CMD="python3 scripts/time_code.py $DVB --batch $BATCH --T 50 --snr 1.0 --variant nms --schedule $sched --reps $REPS --prec $PREC"
  timeout -k 10 240 $CMD > "$D/plain.log" 2>&1 || { echo "$sched plain run failed"; tail -3 "$D/plain.log"; exit 1; }
  tail -1 "$D/plain.log"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$D/stats" -o run --output-format csv -- $CMD \
    > "$D/stats.log" 2>&1 || { echo "$sched stats failed"; tail -3 "$D/stats.log"; exit 1; }
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set -d "$D/p$i" -o pmc --output-format csv -- $CMD \
      > "$D/p$i.log" 2>&1 || { echo "$sched pass $i failed"; tail -3 "$D/p$i.log"; exit 1; }
  done
  echo "$sched: $i passes"
done
echo done
