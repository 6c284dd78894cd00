#!/bin/bash
# Round-2 profiling of the amp-bf16 default bench (GPU box, repo root): kernel trace of the timed
# steps (markers), then one rocprofv3 --pmc pass per counter group, each under its own hard limit.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcb
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bf16 -o trace -- \
    python bench.py --steps 20 --warmup 10 --no-cpu-baseline --markers > gpurun_out/prof_bf16.log 2>&1
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmcb/$name -o $name -- \
      python bench.py --steps 3 --warmup 2 --no-cpu-baseline --markers > gpurun_out/pmcb/$name.log 2>&1
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run mfma SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY
