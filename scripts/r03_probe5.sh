#!/bin/bash
# ping-pong mode 2 (dataflow counters, no interval barriers): parity, A/B vs mode 0
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p5; mkdir -p $O
LDPC_PP_MODE=2 timeout -k 10 120 python -u scripts/pp_check.py > $O/pp_check2.txt 2>&1; rc=$?
cat $O/pp_check2.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_multi.sh 2 "LDPC_ROWS=pp LDPC_PP_MODE=0" "LDPC_ROWS=pp LDPC_PP_MODE=2" -- --no-secondary --steps 5 --warmup 1 || exit 1
