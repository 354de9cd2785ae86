#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p15; mkdir -p $O
PYTEST_TARGETS="tests/test_layered.py tests/test_sharded_gpu.py" RUN_TAG=r03p15 bash scripts/gpu_tests.sh || exit 1
timeout -k 10 900 python -u scripts/config3_sweep.py $O/config3.jsonl > $O/config3.log 2>&1 || { tail -5 $O/config3.log; exit 1; }
python3 -c "
import json
for l in open('$O/config3.jsonl'):
    d=json.loads(l)
    print(d['precision'], d['ebn0_db'], 'frames', d['frames'], 'decoded', d['frames_decoded'], 'rounds', d['rounds'], 's %.3f'%d['seconds'], 'decoded %.0f'%d['sweep_mbit_s_decoded'], 'kernel %.0f Mbit/s %.1f ms'%(d['kernel_mbit_s'], d['ms_per_batch']), 'TB/s %.2f frac %.2f'%(d['achieved_tb_s'], d['frac_of_ic_gather']), 'ovh %.3f'%d['driver_overhead'])
"
bash scripts/ab_multi.sh 2 "LDPC_ROWS=pp" "LDPC_ROWS=pp LDPC_LIB=ppintprem" "LDPC_ROWS=pp LDPC_LIB=ppnofence" -- --no-secondary --steps 5 --warmup 1
