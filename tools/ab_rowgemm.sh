#!/bin/bash
# A/B of the row-streaming GEMM's rows per wave iteration (exp/lib_ni1.so, lib_ni4.so vs the default 2):
# the rowgemm kernel tests on each variant, then alternating 20/5 bench lines.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/rg
for v in ni1 ni4; do
  CTR_LIB_PATH=$PWD/exp/lib_$v.so timeout -k 10 120 python -u -m pytest tests/test_gpu_kernels.py -k rowgemm -q --timeout 120 --timeout-method thread > gpurun_out/rg/test_$v.log 2>&1
done
timeout -k 10 600 bash tools/kexp_bench.sh ni1 ni4 base ni1 ni4 > gpurun_out/rg/ab.log 2>&1
