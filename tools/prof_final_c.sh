#!/bin/bash
# Round-2 re-entry measurement (GPU box, repo root): the colsum kernel tests, the GPU suite, smoke, the
# default bench line (100 timed steps + CPU baseline), the driver's 20/5 line, and the 20/5 step A/B against
# exp/lib_old.so (the previous colsum).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/fin
timeout -k 10 120 python -u -m pytest tests/test_gpu_kernels.py -k "colsum or wgrad" -q --timeout 120 --timeout-method thread > gpurun_out/fin/colsum_test.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/fin/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1
timeout -k 10 240 python bench.py > gpurun_out/fin/bench_n1_final.log 2>&1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fin/bench_n1_s20.log 2>&1
timeout -k 10 300 bash tools/kexp_bench.sh old v4b v4c > gpurun_out/fin/ab_colsum.log 2>&1
