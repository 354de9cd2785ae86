#!/bin/bash
# Round-3 close, part B: headline kernel stats + HBM/SQ PMC, EMS profile and SNR rates.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03b_close; mkdir -p $O
RUN_TAG=r03b_close_prof BENCH_ARGS="--no-secondary" bash scripts/profile_round.sh || exit 1
RUN_TAG=r03b_close_ems bash scripts/profile_ems.sh || exit 1
timeout -k 10 300 python3 scripts/bench_ems.py --ebn0 1.0 1.5 2.0 2.5 --steps 3 > $O/bench_ems.jsonl 2>&1 || { tail -5 $O/bench_ems.jsonl; exit 1; }
echo done
