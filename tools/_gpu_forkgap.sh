#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/t -o t -- python tools/fork_gap_probe.py > $O/probe.log 2>&1
f=$(ls $O/t/*kernel_trace.csv | head -n 1)
python tools/fork_gap_summary.py $f | tee $O/summary.txt
rm -f $O/t/*kernel_trace.csv
