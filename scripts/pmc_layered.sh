#!/bin/bash
# PMC of the layered DVB-S2 kernel (config 3): SQ occupancy/issue counters,
# Infinity-Cache/L2 hits and HBM bytes, one counter group per rocprofv3 pass.
# PREC=f64|f32.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-pmc_layered}
mkdir -p "$OUT"
DVB=$(python3 -c "import sys; sys.path.insert(0, 'tests'); from conftest import code_path; print(code_path('dvbs2_1_2.alist'))")
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_ANY" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o pmc --output-format csv -- \
    python3 scripts/time_code.py "$DVB" --batch 1024 --T 50 --snr 1.0 --variant nms --schedule layered --reps 1 --prec ${PREC:-f64} \
    > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$OUT/p$i.log"; exit 1; }
  tail -1 "$OUT/p$i.log"
done
echo done
