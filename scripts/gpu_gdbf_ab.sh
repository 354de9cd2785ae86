#!/bin/bash
# gdbf_rows A/B (config 4: SMNGDBF, N=1944, T=100, 3.5 dB, 65 536 frames): the
# default library against lib/variants/libldpc_hip_$VARIANT.so, fp32 and fp64,
# two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=${VARIANT:-h0}
O=gpurun_out/gdbf_ab_$V; mkdir -p $O
T="python scripts/time_code.py codes/80211n_1944_r12.alist --batch 65536 --T 100 --decoder gdbf --reps 3 --snr 3.5"
for r in 1 2; do
  for p in f32 f64; do
    timeout -k 10 300 $T --prec $p > $O/def_${p}_$r.log 2>&1 || exit 1; echo "def $p $(tail -1 $O/def_${p}_$r.log | cut -c60-110)"
    LDPC_LIB=$V timeout -k 10 300 $T --prec $p > $O/${V}_${p}_$r.log 2>&1 || exit 1; echo "$V $p $(tail -1 $O/${V}_${p}_$r.log | cut -c60-110)"
  done
done
