#!/bin/bash
# bp_rows occupancy A/B (fp32, N=1944, T=50, 16 384 frames, 2.0 dB): default vs lib/variants/libldpc_hip_bpw8.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/bp_ab; mkdir -p $O
T="python scripts/time_code.py codes/80211n_1944_r12.alist --batch 16384 --T 50 --variant bp --snr 2.0 --reps 3"
for r in 1 2; do
  timeout -k 10 300 $T > $O/def_$r.log 2>&1 || exit 1; echo "def $(tail -1 $O/def_$r.log | cut -c60-110)"
  LDPC_LIB=bpw8 timeout -k 10 300 $T > $O/w8_$r.log 2>&1 || exit 1; echo "w8 $(tail -1 $O/w8_$r.log | cut -c60-110)"
done
