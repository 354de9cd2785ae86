#!/bin/bash
# Round-3 probe: shader clock under load; ping-pong kernel parity; bench A/B
# (k_rows_fast vs k_rows_pp, both prev modes); one block per CU for rows_fast.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p2; mkdir -p $O
timeout -k 10 120 hipcc --offload-arch=gfx950 -O3 -o /tmp/clock_probe scripts/clock_probe.hip 2>/dev/null || exit 1
timeout -k 10 60 /tmp/clock_probe > $O/clock.txt 2>&1 || exit 1
cat $O/clock.txt
timeout -k 10 300 python -u scripts/pp_check.py > $O/pp_check.txt 2>&1; rc=$?
cat $O/pp_check.txt; [ $rc -eq 0 ] || exit $rc
b() { # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 10 --warmup 2 > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$n.json').read().splitlines()[-1]); print('$n', round(d['value'],1), 'Mbit/s', round(d['roofline']['avg_kernel_ms'],3), 'ms', d['kernel_info']['kernel'], 'ferr', d['fer']['frame_err'])"
}
b fast LDPC_ROWS=fast
b pp LDPC_ROWS=pp
b pp_lds LDPC_ROWS=pp LDPC_PP_PREV=lds
b fast2 LDPC_ROWS=fast
b pp2 LDPC_ROWS=pp
b pp_lds2 LDPC_ROWS=pp LDPC_PP_PREV=lds
b fast_bpc1 LDPC_ROWS=fast LDPC_FAST_BPC=1
