# FFN backward variants (exp/lib_<name>.so): isolated kbench (norm-fused, bf16) and the default bench's step
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L="$PWD/exp/lib_$v.so"; fi
  echo "== $v"; CTR_LIB_PATH=$L python tools/kbench.py --which ffn --bf16 --norms --iters 20 || exit 1
  CTR_LIB_PATH=$L python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_$v.json || exit 1
  python -c "
import json; d = json.load(open('gpurun_out/b_$v.json'))
k = d['kernels']; print(d['ms_per_step'], {n: k[n]['avg_launch_ms'] for n in ('ctr_ffn_bwd_norms', 'ctr_ffn_fwd')})"
done
