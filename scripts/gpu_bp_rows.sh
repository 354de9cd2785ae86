#!/bin/bash
# bp_rows vs the generic BP kernel: BP parity tests (and the BP CLI's), then
# timing of both (802.11n N=1944, T=50, 16 384 frames, 2.0 dB) in fp32 and fp64
# and kernel-trace stats of the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN_TAG:-bp_rows}
mkdir -p "$OUT"
step() { local name=$1 lim=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest 600 python -u -m pytest tests/test_bp.py tests/test_cli.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bp or BP"
T="python scripts/time_code.py codes/80211n_1944_r12.alist --batch 16384 --T 50 --variant bp --snr 2.0 --reps 3"
step rows_f32 300 $T
LDPC_BP_KERNEL=generic step generic_f32 300 $T
step rows_f64 300 $T --prec f64
LDPC_BP_KERNEL=generic step generic_f64 300 $T --prec f64
step stats 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 scripts/time_code.py codes/80211n_1944_r12.alist --batch 16384 --T 50 --variant bp --snr 2.0 --reps 2
echo "done $(date +%T)"
