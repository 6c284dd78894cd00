#!/bin/bash
# Side-stream forks merged (CTR_FORK_MERGE=1, default) vs one fork per side block (=0): GPU suite with the merge,
# then same-box bench pairs (cfg2 x3, cfg4 x1) and the fork probe.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -n 30 $O/gputest.log; exit 1; }
tail -n 1 $O/gputest.log
for i in 1 2 3; do
  CTR_FORK_MERGE=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab_off.log 2>&1
  CTR_FORK_MERGE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab_on.log 2>&1
done
CTR_FORK_MERGE=0 timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline >> $O/ab4_off.log 2>&1
CTR_FORK_MERGE=1 timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline >> $O/ab4_on.log 2>&1
