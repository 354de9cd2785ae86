#!/bin/bash
# Scheduler strategies beyond the ping-pong kernel: EMS (max-memory-clause, max-ilp) at
# 2.0 dB and the fp32 row kernel (max-memory-clause), A/B 2 rounds each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${RUN_TAG:-r03p33}; mkdir -p $O
for r in 1 2; do
  for lib in default emsclause emsilp; do
    if [ $lib = default ]; then unset LDPC_LIB; else export LDPC_LIB=$lib; fi
    timeout -k 10 200 python3 scripts/bench_ems.py --ebn0 2.0 --steps 3 > $O/$lib-$r.jsonl 2> $O/$lib-$r.err || { tail -5 $O/$lib-$r.err; exit 1; }
    python3 -c "
import json
for l in open('$O/$lib-$r.jsonl'):
    d=json.loads(l); print('$lib', d['ebn0_db'], round(d['kernel_ms'],3), 'ms', round(d['coded_mbit_s_kernel']), 'Mbit/s')"
  done
done
unset LDPC_LIB
bash scripts/ab_multi.sh 2 "LDPC_ROWS=pp" "LDPC_ROWS=pp LDPC_LIB=rowsclause" -- --precision f32 --steps 5 --warmup 1 --live-pmc off
