#!/bin/bash
# Spill-free ping-pong kernel: row fence, wave priorities and row-1 prefetch re-measured (A/B, 3 rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=("LDPC_ROWS=pp")
for n in ppnofence ppprio1 ppprio3 ppnopf; do A+=("LDPC_ROWS=pp LDPC_LIB=$n"); done
bash scripts/ab_multi.sh 3 "${A[@]}" -- --no-secondary --steps 5 --warmup 1 --live-pmc off
