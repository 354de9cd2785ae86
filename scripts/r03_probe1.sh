#!/bin/bash
# Round-3 probe: shader clock under load, headline bench at HEAD, one block per CU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03p1
timeout -k 10 120 hipcc --offload-arch=gfx950 -O3 -o /tmp/clock_probe scripts/clock_probe.hip 2>/dev/null || exit 1
timeout -k 10 60 /tmp/clock_probe > gpurun_out/r03p1/clock.txt 2>&1 || exit 1
cat gpurun_out/r03p1/clock.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 10 --warmup 2 > gpurun_out/r03p1/bench.json 2> gpurun_out/r03p1/bench.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r03p1/bench.json').read().splitlines()[-1]); print('head', d['value'], d['roofline']['avg_kernel_ms'])"
LDPC_FAST_BPC=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 5 --warmup 1 > gpurun_out/r03p1/bench_bpc1.json 2> gpurun_out/r03p1/bench_bpc1.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r03p1/bench_bpc1.json').read().splitlines()[-1]); print('bpc1', d['value'], d['roofline']['avg_kernel_ms'])"
