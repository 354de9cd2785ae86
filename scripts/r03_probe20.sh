#!/bin/bash
# EMS phase ablations (timing only, early stop off, T=20): which phase holds the time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p20; mkdir -p $O
for lib in default emsexp1 emsexp2 emsexp3; do
  if [ $lib = default ]; then unset LDPC_LIB; else export LDPC_LIB=$lib; fi
  timeout -k 10 200 python3 scripts/bench_ems.py --ebn0 2.0 --steps 3 --no-early-stop > $O/$lib.jsonl 2> $O/$lib.err || { tail -5 $O/$lib.err; exit 1; }
  python3 -c "
import json
for l in open('$O/$lib.jsonl'):
    d=json.loads(l); print('$lib', d['ebn0_db'], round(d['kernel_ms'],2), 'ms', round(d['coded_mbit_s_kernel']), 'Mbit/s iters', d['avg_iters'])"
done
