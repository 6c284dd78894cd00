#!/bin/bash
# Confirmation of the final issue order: GPU suite, smoke, the driver's 20/5 line and the default line.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/fe
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/fe/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fe/smoke.log 2>&1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fe/bench_n1_s20.log 2>&1
timeout -k 10 240 python bench.py > gpurun_out/fe/bench_n1.log 2>&1
