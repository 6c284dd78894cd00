#!/bin/bash
# K > 64 attention backward with the row-statistics loads hoisted before the staging: attention tests with the
# variant library, then cfg4 (K = 148) and cfg3 (K = 100) A/B, two pairs each
set -e
mkdir -p gpurun_out/r05j
CTR_LIB_PATH=$PWD/exp/lib_rs.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_amp.py -m gpu -x -q --timeout 300 --timeout-method thread -k "attn or k148 or cfg3 or cfg4" > gpurun_out/r05j/tests.log 2>&1 || { tail -n 40 gpurun_out/r05j/tests.log; exit 1; }
tail -n 2 gpurun_out/r05j/tests.log
for i in 1 2; do
  for c in cfg4 cfg3; do
    timeout -k 10 200 python bench.py --config $c --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/r05j/${c}_base_$i.log 2>&1
    CTR_LIB_PATH=$PWD/exp/lib_rs.so timeout -k 10 200 python bench.py --config $c --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/r05j/${c}_rs_$i.log 2>&1
    echo "$c base $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05j/${c}_base_$i.log | head -1) $(grep -o '"ctr_attn_bwd_bf": {"calls[^}]*}' gpurun_out/r05j/${c}_base_$i.log) rs $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05j/${c}_rs_$i.log | head -1) $(grep -o '"ctr_attn_bwd_bf": {"calls[^}]*}' gpurun_out/r05j/${c}_rs_$i.log)"
  done
done
