#!/bin/bash
# Ping-pong bit phase: fewer reads in flight per step (VN_U3/VN_U1) A/B, and the
# per-wave stamps of the default and the one-edge-per-step variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${RUN_TAG:-r03p24}; mkdir -p $O
LDPC_LIB=ppu11 timeout -k 10 300 python scripts/pp_check.py > $O/ppcheck_u11.log 2>&1 || { echo "ppcheck failed"; tail -5 $O/ppcheck_u11.log; exit 1; }
echo "ppu11: $(tail -1 $O/ppcheck_u11.log)"
A=("LDPC_ROWS=pp")
for n in ppu11 ppu12 ppu14 ppu22; do A+=("LDPC_ROWS=pp LDPC_LIB=$n"); done
bash scripts/ab_multi.sh 2 "${A[@]}" -- --no-secondary --steps 5 --warmup 1 || exit 1
for v in ppst ppst11; do
  rm -f $O/st.bin
  LDPC_LIB=$v LDPC_ROWS=pp LDPC_STAMPS=$PWD/$O/st.bin timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "== $v"; python scripts/pp_stamps.py $O/st.bin $((128 * 101))
done
