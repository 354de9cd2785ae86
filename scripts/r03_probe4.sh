#!/bin/bash
# ping-pong mode 1 (every thread one row, waves 8-15 also the bit slots): parity, A/B, stamps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p4; mkdir -p $O; rm -f $O/st*.bin
LDPC_PP_MODE=${PPM:-1} timeout -k 10 300 python -u scripts/pp_check.py > $O/pp_check1.txt 2>&1; rc=$?
cat $O/pp_check1.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_multi.sh 2 "LDPC_ROWS=pp LDPC_PP_MODE=0" "LDPC_ROWS=pp LDPC_PP_MODE=1" -- --no-secondary --steps 5 --warmup 1 || exit 1
for m in 0 1; do
LDPC_PP_MODE=$m LDPC_LIB=ppst LDPC_ROWS=pp LDPC_STAMPS=$PWD/$O/st$m.bin timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 > $O/b$m.json 2> $O/b$m.err || { tail -5 $O/b$m.err; exit 1; }
echo "mode $m"; python scripts/pp_stamps.py $O/st$m.bin $((128 * 101)) | head -2
done
