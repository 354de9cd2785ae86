#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03st; mkdir -p $O; rm -f $O/st.bin
LDPC_LIB=ppst LDPC_ROWS=pp LDPC_STAMPS=$PWD/$O/st.bin timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
# 65536 codewords / 256 blocks = 128 pairs per block, 2T+1 = 101 intervals each
python scripts/pp_stamps.py $O/st.bin $((128 * 101))
