#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t -o t -- python bench.py --steps 20 --warmup 10 --no-cpu-baseline --markers > $O/bench.log 2>&1
f=$(ls $O/t/*kernel_trace.csv | head -n 1)
python tools/trace_window.py $f clip_finalize --before 8 --after 4 > $O/win_clip.txt
python tools/trace_window.py $f rowgemm_kernel --before 4 --after 2 --skip 40 --n 3 > $O/win_rowgemm.txt
python tools/trace_window.py $f ffn_bwd_own --before 2 --after 4 --skip 40 --n 2 > $O/win_ffnbwd.txt
rm -f $O/t/*kernel_trace.csv
cat $O/win_clip.txt
