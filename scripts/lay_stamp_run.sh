set -o pipefail
mkdir -p gpurun_out/lay
C=$(python3 -c "import sys; sys.path.insert(0, 'tests'); from conftest import code_path; print(code_path('dvbs2_1_2.alist'))")
LDPC_STAMPS=$PWD/gpurun_out/lay/st.bin timeout -k 10 300 python scripts/time_code.py $C --lib ab/libldpc_hip_laystamp.so --batch 2048 --prec f64 --schedule layered --reps 1 > gpurun_out/lay/t.log 2>&1 && cat gpurun_out/lay/t.log && python scripts/lay_stamps.py gpurun_out/lay/st.bin && timeout -k 10 300 python scripts/time_code.py $C --batch 2048 --prec f64 --schedule layered --reps 2
