#!/bin/bash
# round-5 end validation: the whole GPU suite, smoke, both bench lines, cfg3 / cfg4 lines
set -e
mkdir -p gpurun_out/r05z
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z/gputest.log 2>&1 || { tail -n 40 gpurun_out/r05z/gputest.log; exit 1; }
tail -n 2 gpurun_out/r05z/gputest.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z/smoke.log 2>&1
tail -n 1 gpurun_out/r05z/smoke.log
bash tools/profile.sh r05z bench cfgs
grep -ho '"value": [0-9.]*, "unit": "samples/s"\|"ms_per_step": [0-9.]*, "higher' gpurun_out/r05z/bench_*.log
timeout -k 10 120 python tools/kbench.py --which rowgemm --B 4096 --K 148 --D 64 --bf16 --iters 20 > gpurun_out/r05z/kbench_rowbf.log 2>&1 && cat gpurun_out/r05z/kbench_rowbf.log
