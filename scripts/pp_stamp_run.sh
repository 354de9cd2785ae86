#!/bin/bash
# Per-wave s_memtime stamps of the ping-pong kernel (ab/libldpc_hip_ppst.so from
# scripts/build_stamp_variant.sh): work and barrier-wait cycles per interval for each wave group.
# usage: pp_stamp_run.sh TAG [f64|f32] [bench.py args, e.g. --option pp_slots=plain]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}
PREC=${2:-f64}
shift 2 2>/dev/null || shift $#
O=gpurun_out/stamps_$TAG; mkdir -p $O; rm -f $O/st.bin
LDPC_STAMPS=$PWD/$O/st.bin timeout -k 10 300 python bench.py --lib ${STAMP_LIB:-ab/libldpc_hip_ppst.so} --no-cpu-baseline --no-secondary --steps 2 --warmup 1 --live-pmc off --precision $PREC "$@" > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
# 65536 codewords / 256 blocks: 128 fp64 pairs (or 64 steps of two fp32 pairs) per block, 2T+1 = 101 intervals each
STEPS=$([ "$PREC" = f32 ] && echo 64 || echo 128)
python scripts/pp_stamps.py $O/st.bin $((STEPS * 101)) $STEPS | tee $O/stamps.txt
