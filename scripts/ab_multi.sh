#!/bin/bash
# Interleaved A/B bench runs over whole environment settings (one quoted
# "VAR=v VAR2=w" string per arm), ROUNDS rounds in one session.
# usage: ab_multi.sh ROUNDS "ARM1" "ARM2" ... -- [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUNDS=$1; shift
ARMS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ARMS+=("$1"); shift; done
[ $# -gt 0 ] && shift
mkdir -p gpurun_out/ab_multi
for r in $(seq 1 "$ROUNDS"); do
  for i in "${!ARMS[@]}"; do
    arm=${ARMS[$i]}
    out=gpurun_out/ab_multi/arm$i-$r
    env $arm timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $out.json 2> $out.err || { echo "fail [$arm]"; tail -3 $out.err; exit 1; }
    tail -1 $out.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$arm]', round(d['value'],1), 'Mbit/s', round(d['ms_per_step'],3), 'ms', d['kernel_info'], 'ferr', d['fer']['frame_err'])"
  done
done
