set -u
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
B="--steps 6 --warmup 2 --no-cpu-baseline --live-pmc off --no-secondary"
for r in 1 2; do for T in 2 50; do
  timeout -k 10 120 python bench.py $B --T $T > $O/p_$T.json 2>/dev/null || exit 1
  timeout -k 10 120 python bench.py $B --T $T --lib ab/libldpc_hip_nopipe.so > $O/n_$T.json 2>/dev/null || exit 1
  python3 -c "
import json
for n in ('p_$T','n_$T'):
    d=json.loads(open('$O/'+n+'.json').read().splitlines()[-1]); print(n, round(d['roofline']['avg_kernel_ms'],3))"
done; done
