#!/bin/bash
# Round-2 final measurement, part A (GPU box, repo root): GPU test suite, smoke, the default bench line
# (100 timed steps + the CPU baseline) and the driver's 20/5 line.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/fin
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/fin/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1
timeout -k 10 240 python bench.py > gpurun_out/fin/bench_n1_final.log 2>&1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fin/bench_n1_s20.log 2>&1
