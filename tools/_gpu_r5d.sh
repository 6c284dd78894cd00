#!/bin/bash
# wide-row RMSNorm backward (1024 threads) and the D = 64 wave-independent FFN forward: kernel tests + the amp
# suites that run them; cfg4 A/B (this tree vs HEAD's ffn.hip vs the attention forward at 4 waves / SIMD); the
# cfg4 kernel trace
set -e
mkdir -p gpurun_out/r05e
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_amp.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rmsnorm or rowgemm or ffn or amp or bf16" > gpurun_out/r05e/tests.log 2>&1 || { tail -n 40 gpurun_out/r05e/tests.log; exit 1; }
tail -n 2 gpurun_out/r05e/tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/r05e/c4_base_$i.log 2>&1
  CTR_LIB_PATH=$PWD/exp/lib_ffnhead.so timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/r05e/c4_ffnhead_$i.log 2>&1
  CTR_LIB_PATH=$PWD/exp/lib_aw4.so timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/r05e/c4_aw4_$i.log 2>&1
  grep -Ho '"ms_per_step": [0-9.]*, "higher\|"ctr_attn_fwd_bf": {[^}]*}\|"ctr_ffn_fwd": {[^}]*}' gpurun_out/r05e/c4_base_$i.log gpurun_out/r05e/c4_ffnhead_$i.log gpurun_out/r05e/c4_aw4_$i.log
done
bash tools/profile.sh r05e trace4
