#!/bin/bash
# kernel trace of the default bench's timed steps for the idle-gap analysis (tools/gap_summary.py)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gaps -o trace -- \
    python bench.py --steps 20 --warmup 10 --no-cpu-baseline --markers > gpurun_out/prof_gaps.log 2>&1
f=$(ls gpurun_out/prof_gaps/trace_kernel_trace.csv gpurun_out/prof_gaps/*/trace_kernel_trace.csv 2>/dev/null | head -1)
head -1 "$f" > gpurun_out/trace_header.txt
python tools/gap_summary.py "$f" --steps 20 > gpurun_out/gaps.md
python tools/prof_summary.py "$f" --steps 20 > gpurun_out/ktrace.md
