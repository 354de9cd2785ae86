#!/bin/bash
# One parametrised A/B driver for every kernel experiment (it replaces round 3's 35
# one-off scripts/r03_probe*.sh; their arms and results are in profiles/ab_table_r03.md).
#
# Arms are extra arguments of the timed program, one quoted string each (an empty string
# is the product library with its own kernel choice): "--lib ab/libldpc_hip_<name>.so"
# loads a variant build, "--option rows64=fast" sets a kernel-choice option of the
# context (ldpc_ctx_set_option; the library reads no environment). Build variants on
# the CPU side first (and `make clean-ab` afterwards, so they stop travelling):
#
#   scripts/ab.sh build NAME MAKE_TARGET "VFLAGS"        e.g. build p4 ppvariant "-DLDPC_PP_PRIO=4"
#
# then, on the GPU box, interleaved rounds of one workload per mode:
#
#   scripts/ab.sh bench ROUNDS ARM... [-- bench.py args]        the headline bench (min-sum rows)
#   scripts/ab.sh ems   ROUNDS ARM... [-- bench_ems.py args]    GF(16) EMS (config 5)
#   scripts/ab.sh code  ROUNDS CODE ARM... [-- time_code.py args]   any code (e.g. dvbs2_1_2.alist)
#   scripts/ab.sh check ARM...                                  pp_check.py parity under each arm
#
# Each arm runs under its own time limit; a failing arm stops the script (exit 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mode=$1; shift
O=gpurun_out/ab; mkdir -p $O

if [ "$mode" = build ]; then
  make "$2" NAME="$1" VFLAGS="$3" > /tmp/ab_build_$1.log 2>&1 || { tail -5 /tmp/ab_build_$1.log; exit 1; }
  echo "built ab/libldpc_hip_$1.so"
  exit 0
fi

if [ "$mode" = check ]; then
  for arm in "$@"; do
    timeout -k 10 400 python -u scripts/pp_check.py $arm > $O/check.log 2>&1 || { echo "[$arm] parity FAILED"; tail -5 $O/check.log; exit 1; }
    echo "[$arm] $(tail -1 $O/check.log)"
  done
  exit 0
fi

ROUNDS=$1; shift
CODE=""
if [ "$mode" = code ]; then
  CODE=$(python3 -c "import sys; sys.path.insert(0, 'tests'); from conftest import code_path; print(code_path('$1'))"); shift
fi
ARMS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ARMS+=("$1"); shift; done
[ $# -gt 0 ] && shift
for r in $(seq 1 "$ROUNDS"); do
  for i in "${!ARMS[@]}"; do
    arm=${ARMS[$i]}
    out=$O/$mode-arm$i-$r
    case $mode in
      bench)
        timeout -k 10 300 python bench.py --no-cpu-baseline $arm "$@" > $out.json 2> $out.err || { echo "fail [$arm]"; tail -3 $out.err; exit 1; }
        tail -1 $out.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$arm]', round(d['value'],1), 'Mbit/s', round(d['ms_per_step'],3), 'ms', d['kernel_info']['kernel'], 'ferr', d['fer']['frame_err'])" ;;
      ems)
        timeout -k 10 300 python scripts/bench_ems.py $arm "$@" > $out.json 2> $out.err || { echo "fail [$arm]"; tail -3 $out.err; exit 1; }
        python -c "
import json
for l in open('$out.json'):
    d=json.loads(l); print('[$arm]', d['ebn0_db'], 'dB', round(d['kernel_ms'],3), 'ms', round(d['coded_mbit_s_kernel']), 'Mbit/s', d.get('kernel'), 'fer', d['fer'])" ;;
      code)
        timeout -k 10 300 python scripts/time_code.py "$CODE" $arm "$@" > $out.log 2>&1 || { echo "fail [$arm]"; tail -3 $out.log; exit 1; }
        echo "[$arm] $(tail -1 $out.log)" ;;
      *) echo "unknown mode $mode"; exit 2 ;;
    esac
  done
done
