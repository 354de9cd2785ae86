#!/bin/bash
# Flood phase kernels: resident slots per step (check / bit) A/B on DVB-S2,
# decisions compared across variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p16; mkdir -p $O
for prec in f32 f64; do
  for v in "1 2" "2 2" "4 2" "1 4" "2 4" "4 4"; do
    set -- $v
    d=$O/$prec-c$1-b$2; mkdir -p $d
    echo "== $prec check_sps=$1 bit_sps=$2"
    OUT=$d PREC=$prec LDPC_FLOOD_MODE=phase LDPC_FLOOD_SPS_CHECK=$1 LDPC_FLOOD_SPS_BIT=$2 timeout -k 10 200 python3 scripts/flood_phase_check.py > $d/log 2>&1 || { tail -5 $d/log; exit 1; }
    grep -E "batch|trace" $d/log
  done
done
python3 - <<'PY'
import numpy as np, glob
for prec in ("f32", "f64"):
    fs = sorted(glob.glob(f"gpurun_out/r03p16/{prec}-*/flood_d_phase.npy"))
    ref = np.load(fs[0])
    print(prec, "variants", len(fs), "identical decisions:", all(np.array_equal(ref, np.load(f)) for f in fs))
PY
