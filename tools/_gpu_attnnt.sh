#!/bin/bash
# Attention backward with nontemporal dQKV stores (less dirty L2 left at the kernel boundary) vs the default:
# attention suites with the variant, marker traces + gap summaries of both, bench pairs (cfg2 x2, cfg4 x1).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05t; mkdir -p $O
L=$PWD/exp/lib_attnnt.so
CTR_LIB_PATH=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullshape.py -m gpu -x -q -k "attn or attention or full" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for v in base nt; do
  if [ $v = nt ]; then export CTR_LIB_PATH=$L; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o $v -- python bench.py --steps 20 --warmup 10 --no-cpu-baseline --markers > $O/$v.log 2>&1
  python tools/gap_summary.py $O/$v/${v}_kernel_trace.csv --steps 20 --top 8 > $O/gaps_$v.md
  python tools/prof_summary.py $O/$v/${v}_kernel_trace.csv --steps 20 > $O/trace_$v.md 2>&1 || true
  rm -f $O/$v/${v}_kernel_trace.csv
done
unset CTR_LIB_PATH
head -6 $O/gaps_base.md $O/gaps_nt.md
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab.log 2>&1
  CTR_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab_nt.log 2>&1
done
timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline >> $O/ab4.log 2>&1
CTR_LIB_PATH=$L timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline >> $O/ab4_nt.log 2>&1
