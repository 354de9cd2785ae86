#!/bin/bash
# max-memory-clause scheduling of the ping-pong kernel: parity, then A/B (3 rounds) with
# combinations and code shifts (entry nops) to separate the scheduler from code layout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${RUN_TAG:-r03p31}; mkdir -p $O
LDPC_LIB=ppclause timeout -k 10 300 python scripts/pp_check.py > $O/ppcheck.log 2>&1 || { echo "ppcheck failed"; tail -5 $O/ppcheck.log; exit 1; }
echo "ppclause: $(tail -1 $O/ppcheck.log)"
A=("LDPC_ROWS=pp")
for n in ppclause ppclrelax ppclnohrp ppclnoalign ppclnop1 ppclnop3; do A+=("LDPC_ROWS=pp LDPC_LIB=$n"); done
bash scripts/ab_multi.sh 3 "${A[@]}" -- --no-secondary --steps 5 --warmup 1 --live-pmc off
