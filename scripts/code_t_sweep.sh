#!/bin/bash
# Kernel time of one code against the iteration count T (the per-codeword work is the
# intercept). usage: code_t_sweep.sh CODE [time_code.py args]   e.g. dvbs2_1_2.alist --schedule layered --prec f64
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CODE=$1; shift
A=$(python3 -c "import sys; sys.path.insert(0, 'tests'); from conftest import code_path; print(code_path('$CODE'))")
for T in ${TS:-1 10 50}; do
  timeout -k 10 300 python scripts/time_code.py $A --batch 2048 --T $T --snr 1.0 --variant nms --reps 2 "$@" 2>&1 | tail -1 | sed "s/^/T=$T /" || exit 1
done
