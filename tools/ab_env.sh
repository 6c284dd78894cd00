#!/bin/bash
# A/B on one box (tools/ab.sh compares libraries; this compares an env toggle): env "$1" (e.g. CTR_ROWGRAD_GRAPH=0) vs default, $2 alternating pairs of 20-step bench runs
# AB_EVENTS: bench flags for the event bracketing (default "--kernel-events none"; AB_EVENTS= for the bench default)
set -e
for i in $(seq 1 $2); do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-secondary ${AB_EVENTS---kernel-events none} > gpurun_out/abe_base_$i.log 2>&1
  env $1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-secondary ${AB_EVENTS---kernel-events none} > gpurun_out/abe_exp_$i.log 2>&1
done
for i in $(seq 1 $2); do
  echo "base $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abe_base_$i.log) $1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abe_exp_$i.log)"
done
