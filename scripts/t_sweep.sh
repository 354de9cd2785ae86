#!/bin/bash
# Kernel time of the headline workload against the iteration count T (the per-step
# setup -- channel, staging, syndrome, accounting -- is the intercept).
# usage: t_sweep.sh [bench.py args, e.g. --lib ab/libldpc_hip_x.so]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tsweep; mkdir -p $O
for T in ${TS:-1 10 50}; do
  timeout -k 10 120 python bench.py --T $T --no-secondary --no-cpu-baseline --live-pmc off --steps 5 "$@" > $O/t$T.json 2> $O/t$T.err || { tail -3 $O/t$T.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/t$T.json').read().splitlines()[-1]);print('$*', $T, round(d['roofline']['avg_kernel_ms'],4), round(d['ms_per_step'],4))"
done
