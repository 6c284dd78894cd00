#!/bin/bash
# A/B: the attention-backward side work queued after (main-first) or before (main-first-noattn) the
# in-projection input grad; alternating 20/5 bench lines.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/sa
for o in main-first main-first-noattn main-first main-first-noattn main-first main-first-noattn; do
  CTR_SIDE_ORDER=$o timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sa/b_$o.json
  python -c "import json; d = json.load(open('gpurun_out/sa/b_$o.json')); print('order=$o', d['ms_per_step'], d['value'])" >> gpurun_out/sa/summary.txt
done
CTR_SIDE_ORDER=main-first-noattn timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > gpurun_out/sa/parity_noattn.log 2>&1
