#!/bin/bash
# Sweep-driver rate on config 2 (802.11n N=1944, NMS 1.25, T=50) at 1.75 dB with a
# fixed number of rounds (10 x 65536 frames): blocking rounds (--sync) vs rounds
# launched ahead, in fp64 and fp32. Compare with bench.py's kernel rate.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-sweep_rate}
mkdir -p "$OUT"
ALIST=$(python3 -c "from ldpcsimulation_amd import codes; print(codes.ensure_80211n_1944())")
for prec in f64 f32; do
  for mode in sync async; do
    flag=""; [ $mode = sync ] && flag="--sync"
    timeout -k 10 300 python3 -m ldpcsimulation_amd.sweep "$ALIST" --rate 0.5 --snr 1.75 1.75 -T 50 --variant nms \
      --alpha 1.25 --precision $prec --seed 7 --min-frame-errors 1000000000 --max-frames 655360 --json $flag \
      > "$OUT/$prec-$mode.log" 2>&1 || { echo "fail $prec $mode"; tail -5 "$OUT/$prec-$mode.log"; exit 1; }
    echo "$prec $mode: $(grep '^{' "$OUT/$prec-$mode.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['mbit_s'],1), 'Mbit/s', d['frames'], 'frames', round(d['seconds'],3), 's')")"
  done
done
