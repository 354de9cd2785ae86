#!/bin/bash
# Per-wave s_memtime stamps of the ping-pong kernel (lib/variants/libldpc_hip_ppst.so from
# scripts/build_stamp_variant.sh): work and barrier-wait cycles per interval for each wave group.
# usage: pp_stamp_run.sh TAG  (extra environment, e.g. LDPC_PP_ROWS=plain, passes through)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/stamps_${1:-run}; mkdir -p $O; rm -f $O/st.bin
LDPC_LIB=ppst LDPC_STAMPS=$PWD/$O/st.bin timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 --live-pmc off > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
# 65536 codewords / 256 blocks = 128 pairs per block, 2T+1 = 101 intervals each
python scripts/pp_stamps.py $O/st.bin $((128 * 101)) | tee $O/stamps.txt
