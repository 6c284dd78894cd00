#!/bin/bash
# LayerNorm (norm != "rms"): kernel test, then the reference-run tiny_ln fixture through both training paths
set -e
mkdir -p gpurun_out/r05h
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "layernorm or rmsnorm" > gpurun_out/r05h/ln_kernels.log 2>&1 || { tail -n 40 gpurun_out/r05h/ln_kernels.log; exit 1; }
tail -n 2 gpurun_out/r05h/ln_kernels.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "tiny_ln" > gpurun_out/r05h/ln_parity.log 2>&1 || { tail -n 60 gpurun_out/r05h/ln_parity.log; exit 1; }
tail -n 6 gpurun_out/r05h/ln_parity.log
