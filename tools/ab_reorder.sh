#!/bin/bash
# A/B of the side-stream issue order (CTR_SIDE_ORDER=legacy: side-stream grads queued before the main
# stream's next product; default main-first): GPU suite + smoke on the default order, alternating 20/5 bench
# lines, a kernel trace of the timed steps.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/ab/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab/smoke.log 2>&1
for o in legacy main-first legacy main-first legacy main-first; do
  CTR_SIDE_ORDER=$o timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab/b_$o.json
  python -c "import json; d = json.load(open('gpurun_out/ab/b_$o.json')); print('order=$o', d['ms_per_step'], d['value'])" >> gpurun_out/ab/summary.txt
done
timeout -k 10 240 python bench.py > gpurun_out/ab/bench_n1.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/trace -o trace -- \
    python bench.py --steps 20 --warmup 10 --no-cpu-baseline --markers > gpurun_out/ab/trace.log 2>&1
