#!/bin/bash
# Spill-free ping-pong kernel under LLVM scheduler options (timing A/B, 2 rounds), and
# parity of any variant faster than the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=("LDPC_ROWS=pp")
for n in ppilp ppclause pptrk ppnohrp pprelax; do A+=("LDPC_ROWS=pp LDPC_LIB=$n"); done
bash scripts/ab_multi.sh 2 "${A[@]}" -- --no-secondary --steps 5 --warmup 1 --live-pmc off
