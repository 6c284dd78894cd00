#!/bin/bash
# attention backward (K > 64) keep-word prefetch and the pos-bias grad reduction: tests with the variant library,
# cfg4 A/B (base = HEAD attention + new pos-bias; mklpf = + the prefetch; pbhead = HEAD pos-bias), cfg2 pos-bias A/B
set -e
mkdir -p gpurun_out/r05f
CTR_LIB_PATH=$PWD/exp/lib_mklpf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_amp.py -m gpu -x -q --timeout 300 --timeout-method thread -k "attn or pos_bias or k148" > gpurun_out/r05f/tests.log 2>&1 || { tail -n 40 gpurun_out/r05f/tests.log; exit 1; }
tail -n 2 gpurun_out/r05f/tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/r05f/c4_base_$i.log 2>&1
  CTR_LIB_PATH=$PWD/exp/lib_mklpf.so timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/r05f/c4_mklpf_$i.log 2>&1
  CTR_LIB_PATH=$PWD/exp/lib_pbhead.so timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/r05f/c4_pbhead_$i.log 2>&1
  grep -Ho '"ms_per_step": [0-9.]*, "higher\|"ctr_attn_bwd_bf": {"calls[^}]*}' gpurun_out/r05f/c4_base_$i.log gpurun_out/r05f/c4_mklpf_$i.log gpurun_out/r05f/c4_pbhead_$i.log
done
bash tools/ab.sh pbhead 3
