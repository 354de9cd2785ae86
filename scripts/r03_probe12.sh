#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p12; mkdir -p $O
PYTEST_TARGETS="tests/test_sharded_gpu.py" RUN_TAG=r03p12 bash scripts/gpu_tests.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['kernel_info'], d['roofline']['frac'], d['f32']['value'])"
RUN_TAG=r03_flood1 PREC=f32 bash scripts/r03_flood_gaps.sh || exit 1
LDPC_FLOOD_STREAMS=2 RUN_TAG=r03_flood2 PREC=f32 bash scripts/r03_flood_gaps.sh || exit 1
A=("LDPC_ROWS=pp")
for n in bd2 bd4 prio1 prio2 prio3 exp3 exp4 exp5 exp1 nopf; do A+=("LDPC_ROWS=pp LDPC_LIB=pp$n"); done
bash scripts/ab_multi.sh 2 "${A[@]}" -- --no-secondary --steps 5 --warmup 1
