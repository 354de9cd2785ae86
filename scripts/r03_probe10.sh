#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p10; mkdir -p $O
# EMS: parity of the min3 ECN (main library), then old / min3 / packed-add rates at 2.0 dB
timeout -k 10 600 python -u -m pytest tests/test_ems.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/ems_tests.txt 2>&1; rc=$?
tail -3 $O/ems_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for L in emsold "" emspk; do
  LDPC_LIB=$L timeout -k 10 300 python scripts/bench_ems.py --ebn0 2.0 --steps 3 > $O/ems_$L$r.json 2>$O/ems_$L$r.err || { tail -3 $O/ems_$L$r.err; exit 1; }
  echo "ems [$L] $(tail -1 $O/ems_$L$r.json | cut -c1-300)"
done; done
bash scripts/r03_probe9.sh
