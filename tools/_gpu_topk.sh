#!/bin/bash
# top-K backward split over 4 waves per sample: attention/parity subset with the variant, then per-kernel times
# (rocprofv3 --stats) of a short cfg4 run with each library
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05r
CTR_LIB_PATH=$PWD/exp/lib_split.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --deselect tests/test_gpu_parity.py::test_no_cpu_fallback_library_loaded --timeout 300 --timeout-method thread > gpurun_out/r05r/tests.log 2>&1 || { tail -n 30 gpurun_out/r05r/tests.log; exit 1; }
tail -n 1 gpurun_out/r05r/tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05r/base -o base -- python bench.py --config cfg4 --steps 4 --warmup 2 --no-cpu-baseline --kernel-events none > gpurun_out/r05r/base.log 2>&1
CTR_LIB_PATH=$PWD/exp/lib_split.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05r/split -o split -- python bench.py --config cfg4 --steps 4 --warmup 2 --no-cpu-baseline --kernel-events none > gpurun_out/r05r/split.log 2>&1
grep -h "topk_bwd" gpurun_out/r05r/base/base_kernel_stats.csv gpurun_out/r05r/split/split_kernel_stats.csv | cut -c1-200
rm -f gpurun_out/r05r/*/*_kernel_trace.csv
