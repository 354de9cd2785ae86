#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/ab_multi.sh 2 "LDPC_ROWS=pp LDPC_LIB=ppold" "LDPC_ROWS=pp LDPC_LIB=ppcur" "LDPC_ROWS=pp" "LDPC_ROWS=pp LDPC_LIB=ppexp5" "LDPC_ROWS=pp LDPC_LIB=ppexp6" "LDPC_ROWS=pp LDPC_LIB=ppexp7" "LDPC_ROWS=pp LDPC_LIB=ppbd2" "LDPC_ROWS=pp LDPC_LIB=ppbd5" -- --no-secondary --steps 5 --warmup 1
