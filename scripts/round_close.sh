#!/bin/bash
# Round close at HEAD: full GPU suite + smoke, the default bench line (live PMC traffic,
# CPU baseline), then kernel-trace stats and PMC passes of the headline (profile_round.sh).
# usage: round_close.sh TAG   -> gpurun_out/TAG (copy the summaries into profiles/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
O=gpurun_out/$TAG; mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  RUN_TAG=$TAG PYTEST_TIMEOUT=900 bash scripts/gpu_tests.sh || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
  echo "smoke: $(tail -1 $O/smoke.log | cut -c1-200)"
fi
timeout -k 10 600 python bench.py > $O/bench.jsonl 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.jsonl').read().splitlines()[-1]); r=d['roofline']; c=d.get('cpu_baseline',{})
print('bench', round(d['value']), round(d['ms_per_step'],3), 'frac', round(r['frac'],4), 'traffic', r['traffic'], 'f32', round(d['f32']['value']), d['f32']['kernel'], d['f32'].get('traffic'), 'cpu', c.get('value'), c.get('scaling_curve'))"
RUN_TAG=${TAG}_prof BENCH_ARGS="--no-secondary" bash scripts/profile_round.sh || exit 1
echo done
