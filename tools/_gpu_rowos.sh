#!/bin/bash
# Row-grad sort: rocPRIM onesweep forced (merge-sort limit 0) vs the default (merge sort below 1M keys).
# Parity/lazy suites with the variant, per-kernel stats of a cfg2 run with each, then two bench pairs.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05s; mkdir -p $O
L=$PWD/exp/lib_rowos.so
CTR_LIB_PATH=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lazy.py tests/test_gpu_shard.py -m gpu -x -q --deselect tests/test_gpu_parity.py::test_no_cpu_fallback_library_loaded --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base -o base -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-events none > $O/base.log 2>&1
CTR_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/os -o os -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-events none > $O/os.log 2>&1
python tools/sortstats.py $O/base/base_kernel_stats.csv $O/os/os_kernel_stats.csv | tee $O/sortstats.txt
rm -f $O/*/*_kernel_trace.csv
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab.log 2>&1
  CTR_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab_os.log 2>&1
done
grep -ho '"ms_per_step": [0-9.]*' $O/ab.log $O/ab_os.log
