#!/bin/bash
# Round-2 profiling recipe (run on the GPU box from the repo root): bench line, counter list, kernel
# trace of the timed steps (cut at the bench's step markers), cfg4 bench.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 python bench.py --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/bench_cfg2.log 2>&1
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ktrace -o trace -- \
    python bench.py --steps 20 --warmup 10 --no-cpu-baseline --markers > gpurun_out/prof_ktrace.log 2>&1
timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/bench_cfg4.log 2>&1
