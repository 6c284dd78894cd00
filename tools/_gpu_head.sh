#!/bin/bash
# End-of-round confirmation at HEAD: GPU suite, smoke, the default bench line and the driver's 20 + 5.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -n 30 $O/gputest.log; exit 1; }
tail -n 1 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -n 1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_s20.log 2>&1
grep -h '^{' $O/bench.log $O/bench_s20.log | cut -c1-160
