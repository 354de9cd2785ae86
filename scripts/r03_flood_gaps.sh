#!/bin/bash
# DVB-S2 flooding (phase launches): kernel trace of
# scripts/flood_phase_check.py and the launch-boundary gap histogram
# (scripts/kernel_gaps.py). PREC=f32|f64, extra env passed through.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${RUN_TAG:-r03_flood}; mkdir -p $O
OUT=$O PREC=${PREC:-f32} timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 scripts/flood_phase_check.py > $O/check.log 2>&1 || { tail -5 $O/check.log; exit 1; }
cat $O/check.log | grep -v amdgpu.ids
T=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_gaps.py "$T" flood --json $O/gaps.json | head -40
