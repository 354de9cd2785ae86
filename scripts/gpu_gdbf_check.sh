set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g3
timeout -k 10 600 python -u -m pytest tests/test_cli.py -m gpu -x -q --timeout 300 --timeout-method thread -k gdbf > gpurun_out/g3/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/g3/pytest.log; [ $rc -ne 0 ] && exit $rc
for snr in 3.0 3.5 4.0; do timeout -k 10 120 python scripts/time_code.py tests/golden/codes/80211n_1944_r12.alist --decoder gdbf --batch 65536 --T 100 --snr $snr --reps 2 || exit 1; done
timeout -k 10 120 python scripts/time_code.py tests/golden/codes/80211n_1944_r12.alist --decoder gdbf --batch 65536 --T 100 --snr 3.5 --reps 2 --prec f64 || exit 1
