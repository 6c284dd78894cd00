#!/bin/bash
# Round-2 closing lines of the final build: cfg3 / cfg4 bench lines (parity configs) and the default line.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/fd
timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/fd/bench_cfg4.log 2>&1
timeout -k 10 200 python bench.py --config cfg3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/fd/bench_cfg3.log 2>&1
timeout -k 10 240 python bench.py > gpurun_out/fd/bench_n1.log 2>&1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fd/bench_n1_s20.log 2>&1
