#!/bin/bash
# bench.py with its live PMC traffic pass (default), then the same command under
# rocprofv3 --kernel-trace --stats (the nested run must skip its own PMC pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${RUN_TAG:-r03live}; mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.jsonl 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.jsonl').read().splitlines()[-1]); r=d['roofline']; print('bench', round(d['value']), d['ms_per_step'], 'frac', round(r['frac'],4), 'traffic', r['traffic'], r['traffic_gbs'], r['traffic_source'], r.get('traffic_detail'), 'cpu', d.get('cpu_baseline',{}).get('value'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/stats.log 2>&1 || { tail -5 $O/stats.log; exit 1; }
grep "\"metric\"" $O/stats.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('nested', d['roofline']['traffic_source'])"
