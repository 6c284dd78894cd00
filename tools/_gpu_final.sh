#!/bin/bash
# round-5 validation on the GPU box: the whole GPU suite, smoke, both bench lines, and the cfg4 attention A/B
set -e
mkdir -p gpurun_out/r05c
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05c/gputest.log 2>&1 || { tail -n 40 gpurun_out/r05c/gputest.log; exit 1; }
tail -n 2 gpurun_out/r05c/gputest.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05c/smoke.log 2>&1
tail -n 1 gpurun_out/r05c/smoke.log
timeout -k 10 240 python bench.py > gpurun_out/r05c/bench_n1.log 2>&1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05c/bench_n1_s20.log 2>&1
grep -o '"value": [0-9.]*, "unit": "samples/s"\|"ms_per_step": [0-9.]*, "higher' gpurun_out/r05c/bench_n1*.log
bash tools/_ab_cfg4.sh aw4
