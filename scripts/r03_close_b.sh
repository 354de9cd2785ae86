#!/bin/bash
# Round-3 evidence, part B: kernel stats of the other decoders (DVB-S2
# flooding with packed messages, layered, BP, NGDBF), layered fp64 PMC, EMS profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
RUN_TAG=r03close_others bash scripts/profile_others.sh || exit 1
RUN_TAG=r03close_layered PREC=f64 bash scripts/pmc_layered.sh || exit 1
RUN_TAG=r03close_ems bash scripts/profile_ems.sh || exit 1
timeout -k 10 300 python3 scripts/bench_ems.py --ebn0 1.0 1.5 2.0 2.5 --steps 3 > gpurun_out/r03close_ems/bench_ems.jsonl 2>&1 || exit 1
echo done
