#!/bin/bash
# DVB-S2 N=64800 global flooding kernel: decoded Mbit/s vs resident codewords per CU
# (LDPC_FLOOD_BPC; unset = the occupancy maximum). 4096 codewords, NMS, T=50, 1.0 dB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-flood_bpc}
mkdir -p "$OUT"
DVB=$(python3 -c "import sys; sys.path.insert(0, 'tests'); from conftest import code_path; print(code_path('dvbs2_1_2.alist'))")
for b in max 1 2 3; do
  if [ "$b" = max ]; then unset LDPC_FLOOD_BPC; else export LDPC_FLOOD_BPC=$b; fi
  echo "=== bpc $b"
  timeout -k 10 120 python3 scripts/time_code.py "$DVB" --batch 4096 --T 50 --snr 1.0 --variant nms --reps 2 \
    > "$OUT/bpc_$b.log" 2>&1 || { echo "bpc $b failed"; tail -5 "$OUT/bpc_$b.log"; exit 1; }
  tail -1 "$OUT/bpc_$b.log"
done
