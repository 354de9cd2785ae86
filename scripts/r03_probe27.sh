#!/bin/bash
# EMS: parity (test_ems.py), then A/B against the previous build (LDPC_LIB=emsold)
# at 1.5 / 2.0 dB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${RUN_TAG:-r03p27}; mkdir -p $O
PYTEST_TARGETS="tests/test_ems.py" RUN_TAG=${RUN_TAG:-r03p27} bash scripts/gpu_tests.sh || exit 1
for r in 1 2; do
  for lib in emsold default; do
    if [ $lib = default ]; then unset LDPC_LIB; else export LDPC_LIB=$lib; fi
    timeout -k 10 200 python3 scripts/bench_ems.py --ebn0 1.5 2.0 --steps 3 > $O/$lib-$r.jsonl 2> $O/$lib-$r.err || { tail -5 $O/$lib-$r.err; exit 1; }
    python3 -c "
import json
for l in open('$O/$lib-$r.jsonl'):
    d=json.loads(l); print('$lib', d['ebn0_db'], round(d['kernel_ms'],3), 'ms', round(d['coded_mbit_s_kernel']), 'Mbit/s', d['kernel'], 'fer', d['fer'])"
  done
done
