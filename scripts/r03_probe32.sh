#!/bin/bash
# Further scheduler options against the max-memory-clause default (A/B, 2 rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=("LDPC_ROWS=pp")
for n in ppitmaxocc ppitminreg ppclbias ppclprio; do A+=("LDPC_ROWS=pp LDPC_LIB=$n"); done
bash scripts/ab_multi.sh 2 "${A[@]}" -- --no-secondary --steps 5 --warmup 1 --live-pmc off
