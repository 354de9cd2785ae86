#!/bin/bash
# Round-3 close at HEAD after the max-memory-clause schedule: full GPU suite + smoke,
# the default bench line (live PMC traffic, CPU baseline), kernel stats + PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03c_close; mkdir -p $O
RUN_TAG=r03c_close PYTEST_TIMEOUT=900 bash scripts/gpu_tests.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log | cut -c1-200)"
timeout -k 10 600 python bench.py > $O/bench.jsonl 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.jsonl').read().splitlines()[-1]); r=d['roofline']; print('bench', round(d['value']), round(d['ms_per_step'],3), 'frac', round(r['frac'],4), 'traffic', r['traffic'], 'GB/s', r['traffic_gbs'], 'cpu', d.get('cpu_baseline',{}).get('value'), 'f32', d['f32']['value'])"
RUN_TAG=r03c_close_prof BENCH_ARGS="--no-secondary" bash scripts/profile_round.sh || exit 1
echo done
