#!/bin/bash
# PMC pass over the config-4 GDBF kernel (gdbf_rows, SMNGDBF N=1944 T=100 3.5 dB, fp32):
# VALU / LDS instruction counts and activity, one counter set per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_gdbf; mkdir -p $OUT
CMD="python3 scripts/time_code.py codes/80211n_1944_r12.alist --batch 65536 --T 100 --snr 3.5 --decoder gdbf --reps 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $OUT/sq -o pmc --output-format csv -- $CMD > $OUT/sq.log 2>&1 || { echo "sq rc=$?"; tail -3 $OUT/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_F32 GRBM_GUI_ACTIVE -d $OUT/sq2 -o pmc --output-format csv -- $CMD > $OUT/sq2.log 2>&1 || { echo "sq2 rc=$?"; tail -3 $OUT/sq2.log; exit 1; }
echo done
