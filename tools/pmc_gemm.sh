#!/bin/bash
set -e
export TMPDIR=/tmp
out=gpurun_out/pmcg; mkdir -p $out
for v in 1 2; do
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/a$v -o a -- python tools/kbench.py --which gemmig --variant $v --iters 2 > $out/a$v.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/b$v -o b -- python tools/kbench.py --which gemmig --variant $v --iters 2 > $out/b$v.log 2>&1
done
