#!/bin/bash
# Layered DVB-S2: GPU parity tests, then an A/B over one environment variable (fp32 and fp64).
# usage: gpu_layered_ab.sh VAR "v1 v2"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lay
timeout -k 10 400 python -u -m pytest tests/test_layered.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/lay/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/lay/pytest.log
[ $rc -ne 0 ] && exit $rc
for prec in f32 f64; do
  bash scripts/ab_code.sh "$1" "$2" 2 dvbs2_1_2.alist --batch 2048 --T 50 --snr 1.0 \
      --schedule layered --reps 2 --prec $prec || exit 1
done
