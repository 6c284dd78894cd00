#!/bin/bash
# A/B of a Python-side change on one box (tools/ab.sh compares libraries, tools/ab_env.sh env toggles):
#   tools/ab_py.sh <file in the tree> <alternative copy of it> <pairs>
# alternating 20-step bench runs with the tree's file ("new") and the alternative ("prev"); the tree's file is restored.
set -e
F=$1
ALT=$2
cp "$F" /tmp/ab_py_new
trap 'cp /tmp/ab_py_new "$F"' EXIT
for i in $(seq 1 $3); do
  cp /tmp/ab_py_new "$F"
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-secondary --kernel-events none > gpurun_out/abp_new_$i.log 2>&1
  cp "$ALT" "$F"
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-secondary --kernel-events none > gpurun_out/abp_prev_$i.log 2>&1
done
for i in $(seq 1 $3); do
  echo "new $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abp_new_$i.log) prev $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abp_prev_$i.log)"
done
