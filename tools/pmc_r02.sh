#!/bin/bash
# Round-2 PMC passes (GPU box, repo root): one counter group per rocprofv3 run, each under its own
# hard time limit; a short bench (markers on) so the summaries can keep the timed steps only.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
run() {  # name config counters...
  local name=$1 cfg=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc/$name -o $name -- \
      python bench.py --config $cfg --steps 3 --warmup 2 --no-cpu-baseline --markers > gpurun_out/pmc/$name.log 2>&1
}
run fetch cfg2 FETCH_SIZE
run write cfg2 WRITE_SIZE
run mfma cfg2 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
run lds cfg2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY
run lds_cfg4 cfg4 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY
run mfma_cfg4 cfg4 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
