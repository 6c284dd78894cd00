# bench A/B of exp/lib_<name>.so variants on one config: step time and the attention / FFN entry timings
cfg=$1; shift
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L="$PWD/exp/lib_$v.so"; fi
  echo "== $v ($cfg)"; CTR_LIB_PATH=$L python bench.py --config $cfg --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/c_$v.json || exit 1
  python -c "
import json; d = json.load(open('gpurun_out/c_$v.json'))
k = d['kernels']; print(d['ms_per_step'], {n: k[n]['avg_launch_ms'] for n in k if 'attn' in n or 'ffn' in n})"
done
