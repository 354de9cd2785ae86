set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lay1; rm -f gpurun_out/lay1/time.log
D=tests/golden/codes/.cache/dvbs2_1_2.alist
timeout -k 10 300 python -u -m pytest tests/test_layered.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/lay1/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/lay1/pytest.log
[ $rc -ge 124 ] && exit $rc
for s in flooding layered; do timeout -k 10 120 python scripts/time_code.py $D --batch 2048 --T 50 --snr 1.0 --schedule $s --reps 2 >> gpurun_out/lay1/time.log 2>&1 || exit 1; done
for b in 2; do LDPC_LAYERED_BPC=$b timeout -k 10 120 python scripts/time_code.py $D --batch 2048 --T 50 --snr 1.0 --schedule layered --reps 2 >> gpurun_out/lay1/time.log 2>&1 || exit 1; echo bpc=$b >> gpurun_out/lay1/time.log; done
timeout -k 10 120 python scripts/time_code.py tests/golden/codes/80211n_1944_r12.alist --batch 65536 --T 50 --snr 1.5 --schedule layered --reps 2 >> gpurun_out/lay1/time.log 2>&1
cat gpurun_out/lay1/time.log
