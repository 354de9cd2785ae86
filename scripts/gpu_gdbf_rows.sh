#!/bin/bash
# gdbf_rows vs the generic GDBF kernel: parity tests, then config-4 timing
# (SMNGDBF, 802.11n N=1944, T=100, 65 536 frames) of both kernels, of the
# occupancy variants (lib/variants/libldpc_hip_w5/w6.so, when built) and of
# fp64, and kernel-trace stats of the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-gdbf_rows}
mkdir -p "$OUT"
step() { local name=$1 lim=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest 600 python -u -m pytest tests/test_gdbf.py -m gpu -x -q --timeout 300 --timeout-method thread
fi
T="python scripts/time_code.py codes/80211n_1944_r12.alist --batch 65536 --T 100 --decoder gdbf --reps 3"
for r in 1 2; do
  step rows_f32_$r 300 $T --snr 3.5
  for v in ${VARIANTS:-w4}; do
    [ -f ldpcsimulation_amd/lib/variants/libldpc_hip_$v.so ] && LDPC_LIB=$v step ${v}_f32_$r 300 $T --snr 3.5
  done
done
LDPC_GDBF_KERNEL=generic step generic_f32 300 $T --snr 3.5
step rows_f64 300 $T --snr 3.5 --prec f64
LDPC_GDBF_KERNEL=generic step generic_f64 300 $T --snr 3.5 --prec f64
step rows_f32_3.0 300 $T --snr 3.0
step rows_f32_4.0 300 $T --snr 4.0
step stats 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 scripts/time_code.py codes/80211n_1944_r12.alist --batch 65536 --T 100 --snr 3.5 --decoder gdbf --reps 2
echo "done $(date +%T)"
