set -e
for i in 1 2; do
  timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/c4_base_$i.log 2>&1
  CTR_LIB_PATH=$PWD/exp/lib_$1.so timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/c4_exp_$i.log 2>&1
done
for i in 1 2; do python3 - "$i" <<'PY'
import json,sys
i=sys.argv[1]
for k in ("base","exp"):
    d=json.loads(open(f"gpurun_out/c4_{k}_{i}.log").read().strip().split("\n")[-1])
    ks={n:v["avg_launch_ms"] for n,v in d["kernels"].items() if "attn" in n}
    print(k, d["ms_per_step"], ks)
PY
done
