#!/bin/bash
# EMS kernel time against the iteration count (early stop off), and the early-stop run:
# the per-codeword work (channel, initial messages, accounting) is the intercept.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for T in 1 5 20; do
  timeout -k 10 120 python scripts/bench_ems.py --ebn0 2.0 --steps 2 --batch 16384 --T $T --no-early-stop > gpurun_out/ems_t$T.json 2>&1 || { tail -3 gpurun_out/ems_t$T.json; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ems_t$T.json').read().splitlines()[-1]);print($T, round(d['kernel_ms'],4), d['avg_iters'])"
done
timeout -k 10 120 python scripts/bench_ems.py --ebn0 2.0 --steps 2 --batch 16384 > gpurun_out/ems_es.json 2>&1 && python -c "import json;d=json.loads(open('gpurun_out/ems_es.json').read().splitlines()[-1]);print('es', round(d['kernel_ms'],4), d['avg_iters'], d['coded_mbit_s_kernel'])"
