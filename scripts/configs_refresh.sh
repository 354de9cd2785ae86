#!/bin/bash
# One pass over the secondary configs at HEAD (kernel rates; results to gpurun_out/configs/):
# config 3 DVB-S2 (layered and flooding, fp64 and fp32), config 4 SMNGDBF on N=1944,
# config 5 GF(16) EMS at 1.5 / 2.0 / 2.5 dB, config 1 PEG 1008.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/configs; mkdir -p $O
cp() { python3 -c "import sys; sys.path.insert(0, 'tests'); from conftest import code_path; print(code_path('$1'))"; }
DVB=$(cp dvbs2_1_2.alist); N1944=$(cp 80211n_1944_r12.alist); PEG=$(cp PEGReg504x1008.alist)
run() { local n=$1; shift; timeout -k 10 300 python "$@" > $O/$n.log 2>&1 || { echo "fail $n"; tail -3 $O/$n.log; exit 1; }; echo "$n: $(tail -1 $O/$n.log | cut -c1-260)"; }
run c3_layered_f64 scripts/time_code.py $DVB --batch 2048 --T 50 --snr 1.0 --prec f64 --schedule layered --reps 2
run c3_layered_f32 scripts/time_code.py $DVB --batch 2048 --T 50 --snr 1.0 --prec f32 --schedule layered --reps 2
run c3_flood_f64 scripts/time_code.py $DVB --batch 2048 --T 50 --snr 1.0 --prec f64 --reps 2
run c3_flood_f32 scripts/time_code.py $DVB --batch 2048 --T 50 --snr 1.0 --prec f32 --reps 2
run c4_gdbf_f32 scripts/time_code.py $N1944 --decoder gdbf --batch 65536 --T 100 --snr 3.5 --prec f32 --reps 2
run c4_gdbf_f64 scripts/time_code.py $N1944 --decoder gdbf --batch 65536 --T 100 --snr 3.5 --prec f64 --reps 2
run c5_ems scripts/bench_ems.py --ebn0 1.5 2.0 2.5 --steps 3 --batch 16384
run c1_peg_f64 scripts/time_code.py $PEG --batch 65536 --T 10 --snr 2.0 --variant ms --prec f64 --reps 2
