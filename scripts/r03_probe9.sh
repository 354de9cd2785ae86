#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=()
for n in n0 n1 n2 n3 a32n0 a32n1 a32n2 a32n3; do A+=("LDPC_ROWS=pp LDPC_LIB=pp$n"); done
bash scripts/ab_multi.sh 2 "${A[@]}" -- --no-secondary --steps 5 --warmup 1
