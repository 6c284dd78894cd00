#!/bin/bash
# cfg4 PMC passes + kernel trace, summarised on the box (the raw CSVs exceed gpurun's 64 MiB copy-back)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/profile.sh r05q pmc4 trace4
O=gpurun_out/r05q
mkdir -p $O/pm gpurun_out/r05q_sum
for p in fetch write valu mops lds; do
  mkdir -p $O/pm/$p
  cp $O/pmc_${p}_cfg4/${p}_cfg4_counter_collection.csv $O/pm/$p/${p}_counter_collection.csv
done
python tools/prof_summary.py $O/trace4/trace4_kernel_trace.csv --steps 6 > gpurun_out/r05q_sum/kernel_trace_cfg4_final.md
python tools/stream_summary.py $O/trace4/trace4_kernel_trace.csv --steps 6 > gpurun_out/r05q_sum/streams_cfg4_final.md
python tools/pmc_summary.py $O/pm --passes fetch write valu mops lds --trace-md gpurun_out/r05q_sum/kernel_trace_cfg4_final.md --title "PMC counters per kernel, cfg4 (D=64, K=148, 4 layers, amp bf16), timed steps, end of round 5" > gpurun_out/r05q_sum/pmc_cfg4_final.md
cp $O/trace4/trace4_kernel_stats.csv gpurun_out/r05q_sum/kernel_stats_cfg4_final.csv
rm -rf $O
ls -la gpurun_out/r05q_sum
