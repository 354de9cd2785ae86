#!/bin/bash
# Flood phase with packed messages: resident slots K (LDPC_FLOOD_RESIDENT) sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p18; mkdir -p $O
for prec in f32 f64; do
  if [ $prec = f32 ]; then KS="96 112 128 144"; else KS="64 80 96 112 128"; fi
  for k in $KS; do
    d=$O/$prec-$k; mkdir -p $d
    echo "== $prec K=$k"
    if [ $k = 0 ]; then unset LDPC_FLOOD_RESIDENT; else export LDPC_FLOOD_RESIDENT=$k; fi
    OUT=$d PREC=$prec BATCH=4096 timeout -k 10 200 python3 scripts/flood_phase_check.py > $d/log 2>&1 || { tail -5 $d/log; exit 1; }
    grep -E "batch" $d/log
  done
done
