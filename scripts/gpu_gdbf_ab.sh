set -u
export TMPDIR=/tmp
O=gpurun_out/gdbf_ab7; mkdir -p $O
T="python scripts/time_code.py codes/80211n_1944_r12.alist --batch 65536 --T 100 --decoder gdbf --reps 3 --snr 3.5"
for r in 1 2; do
  timeout -k 10 300 $T > $O/def_f32_$r.log 2>&1 || exit 1; echo "def f32 $(tail -1 $O/def_f32_$r.log | cut -c60-120)"
  LDPC_LIB=w8 timeout -k 10 300 $T > $O/w8_f32_$r.log 2>&1 || exit 1; echo "w8 f32 $(tail -1 $O/w8_f32_$r.log | cut -c60-120)"
  timeout -k 10 300 $T --prec f64 > $O/def_f64_$r.log 2>&1 || exit 1; echo "def f64 $(tail -1 $O/def_f64_$r.log | cut -c60-120)"
  LDPC_LIB=d6 timeout -k 10 300 $T --prec f64 > $O/d6_f64_$r.log 2>&1 || exit 1; echo "d6 f64 $(tail -1 $O/d6_f64_$r.log | cut -c60-120)"
done
timeout -k 10 400 python -u -m pytest tests/test_gdbf.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$? $(tail -1 $O/pytest.log)"
