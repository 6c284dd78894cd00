#!/bin/bash
# A/B cfg4: default library vs exp/lib_$1.so, $2 alternating pairs
set -e
for i in $(seq 1 $2); do
  timeout -k 10 120 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/ab4_base_$i.log 2>&1
  CTR_LIB_PATH=exp/lib_$1.so timeout -k 10 120 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/ab4_exp_$i.log 2>&1
done
for i in $(seq 1 $2); do
  python -c "
import json,sys
for n in ('base','exp'):
    d=[json.loads(l) for l in open(f'gpurun_out/ab4_{n}_$i.log') if l.startswith('{')][-1]
    print(n, d['ms_per_step'], d['kernels']['ctr_ffn_bwd_norms']['avg_launch_ms'], end='  ')
print()"
done
