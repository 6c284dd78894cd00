#!/bin/bash
# DARE lazy update on the side stream: the lazy / parity / full-shape tests, then a cfg2 A/B (3 alternating pairs)
set -e
mkdir -p gpurun_out/r05i
timeout -k 10 900 python -u -m pytest tests/test_gpu_lazy.py tests/test_gpu_parity.py tests/test_gpu_fullshape.py tests/test_gpu_train.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05i/tests.log 2>&1 || { tail -n 40 gpurun_out/r05i/tests.log; exit 1; }
tail -n 2 gpurun_out/r05i/tests.log
for i in 1 2 3; do
  timeout -k 10 120 python tools/seq_update_main.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-events none > gpurun_out/r05i/ab_main_$i.log 2>&1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-events none > gpurun_out/r05i/ab_side_$i.log 2>&1
  echo "main $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05i/ab_main_$i.log) side $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05i/ab_side_$i.log)"
done
timeout -k 10 240 python tools/seq_update_main.py > gpurun_out/r05i/ab_main_100.log 2>&1
timeout -k 10 240 python bench.py > gpurun_out/r05i/ab_side_100.log 2>&1
echo "100 steps: main $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05i/ab_main_100.log) side $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05i/ab_side_100.log)"
