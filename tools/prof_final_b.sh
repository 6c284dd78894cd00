#!/bin/bash
# Round-2 final measurement, part B: kernel trace of the timed steps (+ idle-gap attribution), one rocprofv3
# --pmc pass per counter group (each under its own hard limit), cfg3 / cfg4 bench lines.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/fin/pmc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin/trace -o trace -- \
    python bench.py --steps 20 --warmup 10 --no-cpu-baseline --markers > gpurun_out/fin/trace.log 2>&1
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/fin/pmc/$name -o $name -- \
      python bench.py --steps 3 --warmup 2 --no-cpu-baseline --markers > gpurun_out/fin/pmc/$name.log 2>&1
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY
timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/fin/bench_cfg4.log 2>&1
timeout -k 10 200 python bench.py --config cfg3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/fin/bench_cfg3.log 2>&1
