#!/bin/bash
# A/B bench runs over values of one environment variable, interleaved rounds in one session.
# usage: ab_env.sh VAR "v1 v2 ..." ROUNDS [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VAR=$1; VALS=$2; ROUNDS=$3; shift 3
mkdir -p gpurun_out/ab
for r in $(seq 1 $ROUNDS); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab/$VAR-$v-$r.json 2> gpurun_out/ab/$VAR-$v-$r.err || { echo "fail $v"; tail -3 gpurun_out/ab/$VAR-$v-$r.err; exit 1; }
    tail -1 gpurun_out/ab/$VAR-$v-$r.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v', round(d['value'],1), 'Mbit/s', round(d['ms_per_step'],3), 'ms', d['kernel_info'], 'ferr', d['fer']['frame_err'])"
  done
done
