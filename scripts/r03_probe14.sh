#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p14; mkdir -p $O
PYTEST_TARGETS="tests/test_layered.py" RUN_TAG=r03p14 bash scripts/gpu_tests.sh || exit 1
LDPC_LAYERED_THREADS=1024 PYTEST_TARGETS="tests/test_layered.py" RUN_TAG=r03p14b bash scripts/gpu_tests.sh || exit 1
bash scripts/ab_code.sh LDPC_LAYERED_THREADS "512 1024" 2 dvbs2_1_2.alist --batch 2048 --T 50 --snr 1.0 --schedule layered --reps 2 --prec f32 || exit 1
bash scripts/ab_code.sh LDPC_LAYERED_THREADS "512 1024" 2 dvbs2_1_2.alist --batch 2048 --T 50 --snr 1.0 --schedule layered --reps 2 --prec f64 || exit 1
for p in f32 f64; do timeout -k 10 300 python scripts/time_code.py $(python3 -c "import sys; sys.path.insert(0,'tests'); from conftest import code_path; print(code_path('dvbs2_1_2.alist'))") --batch 2048 --T 50 --snr 1.0 --reps 2 --prec $p; done
