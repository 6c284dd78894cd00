# default-bench A/B of exp/lib_<name>.so variants: step time and the lazy-table kernels' timings
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L="$PWD/exp/lib_$v.so"; fi
  echo "== $v"; CTR_LIB_PATH=$L python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_$v.json || exit 1
  python -c "
import json; d = json.load(open('gpurun_out/b_$v.json'))
k = d['kernels']; print(d['ms_per_step'], d['flush_ms'], {n: k[n]['avg_launch_ms'] for n in k if 'lazy' in n or 'qnn' in n})"
done
