#!/bin/bash
# A/B of the pipelined fp64 step (LDPC_PP_PIPE, default) against pp_role's step
# (ab/libldpc_hip_nopipe.so: make ppvariant NAME=nopipe VFLAGS=-DLDPC_PP_PIPE=0), with
# the rows_pp / parity GPU tests first and per-wave stamps of both
# (ab/libldpc_hip_ppst_{pipe,nopipe}.so: scripts/build_stamp_variant.sh [EXTRA=-DLDPC_PP_PIPE=0]).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${RUN_TAG:-abpipe}; mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rows_pp.py tests/test_gpu_parity.py > $O/t.log 2>&1
  rc=$?; tail -3 $O/t.log
  [ $rc -ne 0 ] && exit $rc
fi
B="--steps 10 --warmup 2 --no-cpu-baseline --live-pmc off --no-secondary"
for k in 1 2 3; do
  timeout -k 10 120 python bench.py $B > $O/pipe_$k.json 2>$O/pipe_$k.err || exit 1
  timeout -k 10 120 python bench.py $B --lib ab/libldpc_hip_nopipe.so > $O/nopipe_$k.json 2>$O/nopipe_$k.err || exit 1
  python3 -c "
import json
for n in ('pipe_$k','nopipe_$k'):
    d=json.loads(open('$O/'+n+'.json').read().splitlines()[-1]); print(n, round(d['ms_per_step'],3), round(d['roofline']['avg_kernel_ms'],3), round(d['value']), d['fer']['frame_err'], d['fer']['redecoded_exact_last_launch'])"
done
if [ -f ab/libldpc_hip_ppst_pipe.so ]; then
  for v in pipe nopipe; do
    rm -f $O/st_$v.bin
    LDPC_STAMPS=$PWD/$O/st_$v.bin timeout -k 10 200 python bench.py --lib ab/libldpc_hip_ppst_$v.so --no-cpu-baseline --no-secondary --steps 2 --warmup 1 --live-pmc off > $O/st_$v.json 2> $O/st_$v.err || exit 1
    IV=$([ $v = pipe ] && echo $((128 * 103 + 2)) || echo $((128 * 101)))
    echo "== stamps $v (intervals per block $IV)"; python scripts/pp_stamps.py $O/st_$v.bin $IV | tail -4 | tee $O/stamps_$v.txt
  done
fi
