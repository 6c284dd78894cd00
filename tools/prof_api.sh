#!/bin/bash
# kernel + HIP runtime API trace of the default bench's timed steps (tools/gap_api.py)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/prof_api -o trace -- \
    python bench.py --steps 20 --warmup 10 --no-cpu-baseline --markers > gpurun_out/prof_api.log 2>&1
ls gpurun_out/prof_api
