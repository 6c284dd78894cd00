#!/bin/bash
# bf16 row kernels at D = 64: kernel tests, the amp band tests, cfg4 A/B (fp32 GEMM routing vs rowgemm_bf), then
# the round's full GPU validation
set -e
mkdir -p gpurun_out/r05d
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rowgemm" > gpurun_out/r05d/rowbf_tests.log 2>&1 || { tail -n 40 gpurun_out/r05d/rowbf_tests.log; exit 1; }
tail -n 2 gpurun_out/r05d/rowbf_tests.log
for i in 1 2; do
  timeout -k 10 200 python tools/nobf_rows.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/r05d/c4_old_$i.log 2>&1
  timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/r05d/c4_new_$i.log 2>&1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05d/c4_old_$i.log gpurun_out/r05d/c4_new_$i.log
done
bash tools/_gpu_final.sh
