#!/bin/bash
# Round-3 evidence, part A: full GPU suite, the headline profile (stats + HBM
# and SQ PMC passes of bench.py), then the bench line at HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03close; mkdir -p $O
RUN_TAG=r03close PYTEST_TIMEOUT=900 bash scripts/gpu_tests.sh || exit 1
RUN_TAG=r03close_prof BENCH_ARGS="--no-secondary" bash scripts/profile_round.sh || exit 1
python3 scripts/summarize_profile.py gpurun_out/r03close_prof r03_close_bench k_rows_pp f64 > $O/summ.log 2>&1 || { cat $O/summ.log; exit 1; }
timeout -k 10 600 python3 bench.py > $O/bench.jsonl 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.jsonl | cut -c1-600
