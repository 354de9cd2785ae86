#!/bin/bash
# EMS: symbol c2v cache depth (VD 4 default / 2) and 1024-thread blocks (4 waves per SIMD).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${RUN_TAG:-r03p22}; mkdir -p $O
for r in 1 2; do
  for arm in default noopq t512; do
    unset LDPC_LIB LDPC_EMS_THREADS
    case $arm in
      noopq) export LDPC_LIB=emsnoopq;;
      t512) export LDPC_EMS_THREADS=512;;
    esac
    timeout -k 10 200 python3 scripts/bench_ems.py --ebn0 1.5 2.0 --steps 3 > $O/$arm-$r.jsonl 2> $O/$arm-$r.err || { tail -5 $O/$arm-$r.err; exit 1; }
    python3 -c "
import json
for l in open('$O/$arm-$r.jsonl'):
    d=json.loads(l); print('$arm', d['ebn0_db'], round(d['kernel_ms'],2), 'ms', round(d['coded_mbit_s_kernel']), 'Mbit/s', d['kernel'])"
  done
done
PYTEST_TARGETS="tests/test_ems.py" RUN_TAG=${RUN_TAG:-r03p22} bash scripts/gpu_tests.sh
