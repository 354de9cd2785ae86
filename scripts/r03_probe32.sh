#!/bin/bash
# Further scheduler options against max-memory-clause (A/B, 2 rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=("LDPC_ROWS=pp LDPC_LIB=ppclause")
for n in ppclrelax ppitmaxocc ppitminreg ppclprio ppclbias; do A+=("LDPC_ROWS=pp LDPC_LIB=$n"); done
bash scripts/ab_multi.sh 2 "${A[@]}" -- --no-secondary --steps 5 --warmup 1 --live-pmc off
