#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p13; mkdir -p $O
PYTEST_TARGETS="tests/test_layered.py tests/test_gpu_parity.py" RUN_TAG=r03p13 bash scripts/gpu_tests.sh || exit 1
for st in 1 2; do
  LDPC_FLOOD_STREAMS=$st PREC=f32 OUT=$O timeout -k 10 300 python scripts/flood_phase_check.py > $O/flood$st.log 2>&1 || { tail -3 $O/flood$st.log; exit 1; }
  echo "streams=$st"; grep batch $O/flood$st.log
done
PREC=f64 OUT=$O timeout -k 10 300 python scripts/flood_phase_check.py > $O/flood64.log 2>&1 || exit 1
echo "f64:"; grep batch $O/flood64.log
timeout -k 10 900 python -u scripts/config3_sweep.py $O/config3.jsonl > $O/config3.log 2>&1; rc=$?
cut -c1-400 $O/config3.log; exit $rc
