#!/bin/bash
# rocprofv3 kernel-trace stats of the non-headline decoders (BP, GDBF/NGDBF,
# DVB-S2 flooding and layered), one short timing run each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-others_prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
DVB=$(python3 -c "import sys; sys.path.insert(0, 'tests'); from conftest import code_path; print(code_path('dvbs2_1_2.alist'))")
run() {   # name, args...
  local name=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o "$name" --output-format csv -- \
    python3 scripts/time_code.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; exit 1; }
  tail -1 "$OUT/$name.log"
}
run bp_f32 codes/80211n_1944_r12.alist --batch 16384 --T 50 --snr 1.5 --variant bp --prec f32 --reps 2
run ngdbf codes/80211n_1944_r12.alist --batch 65536 --T 100 --snr 3.5 --decoder gdbf --reps 2
run dvbs2_flood "$DVB" --batch 2048 --T 50 --snr 1.0 --variant nms --reps 2
run dvbs2_layered "$DVB" --batch 2048 --T 50 --snr 1.0 --variant nms --schedule layered --reps 2
run dvbs2_layered_f64 "$DVB" --batch 2048 --T 50 --snr 1.0 --variant nms --schedule layered --reps 2 --prec f64
run dvbs2_flood_f64 "$DVB" --batch 2048 --T 50 --snr 1.0 --variant nms --reps 2 --prec f64
echo done
