#!/bin/bash
# A/B: default library vs exp/lib_$1.so, $2 alternating pairs of 20-step bench runs
set -e
for i in $(seq 1 $2); do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-secondary --kernel-events none > gpurun_out/ab_base_$i.log 2>&1
  CTR_LIB_PATH=exp/lib_$1.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-secondary --kernel-events none > gpurun_out/ab_exp_$i.log 2>&1
done
for i in $(seq 1 $2); do
  echo "base $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_base_$i.log) exp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_exp_$i.log)"
done
