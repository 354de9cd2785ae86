#!/bin/bash
# EMS: symbol-node c2v in registers (default, VD=4) vs re-read (VD=0 variant); EMS tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${RUN_TAG:-r03p19}; mkdir -p $O
for r in 1 2; do
  for lib in emsnopair default; do
    if [ $lib = default ]; then unset LDPC_LIB; else export LDPC_LIB=$lib; fi
    echo "== $lib"
    timeout -k 10 200 python3 scripts/bench_ems.py --ebn0 1.5 2.0 --steps 3 > $O/$lib-$r.jsonl 2> $O/$lib-$r.err || { tail -5 $O/$lib-$r.err; exit 1; }
    python3 -c "
import json
for l in open('$O/$lib-$r.jsonl'):
    d=json.loads(l); print(d['ebn0_db'], round(d['kernel_ms'],2), 'ms', round(d['coded_mbit_s_kernel']), 'Mbit/s', 'iters', round(d['avg_iters'],2), 'fer', d['fer'])"
  done
done
unset LDPC_LIB
PYTEST_TARGETS="tests/test_ems.py" RUN_TAG=${RUN_TAG:-r03p19} bash scripts/gpu_tests.sh
