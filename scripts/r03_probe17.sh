#!/bin/bash
# Flood phase: packed-state messages (default) vs the c2v array; decisions compared.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p17; mkdir -p $O
for prec in f32 f64; do
  for m in c2v packed; do
    for sb in 1 2; do
      d=$O/$prec-$m-$sb; mkdir -p $d
      echo "== $prec msg=$m bit_sps=$sb"
      OUT=$d PREC=$prec LDPC_FLOOD_MODE=phase LDPC_FLOOD_MSG=$m LDPC_FLOOD_SPS_BIT=$sb timeout -k 10 200 python3 scripts/flood_phase_check.py > $d/log 2>&1 || { tail -5 $d/log; exit 1; }
      grep -E "batch|trace" $d/log
    done
  done
done
python3 - <<'PY'
import numpy as np, glob
for prec in ("f32", "f64"):
    fs = sorted(glob.glob(f"gpurun_out/r03p17/{prec}-*/flood_d_phase.npy"))
    ref = np.load(fs[0])
    print(prec, "variants", len(fs), "identical decisions:", all(np.array_equal(ref, np.load(f)) for f in fs))
PY
PYTEST_TARGETS="tests/test_gpu_parity.py" RUN_TAG=r03p17 bash scripts/gpu_tests.sh
