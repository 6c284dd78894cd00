#!/bin/bash
# PMC passes over tools/kbench.py (GPU box, repo root): one counter group per rocprofv3 run, each under
# its own hard limit.  Usage: tools/pmc_kbench.sh <outdir> <kbench args...>
set -e
export TMPDIR=/tmp
out=$1; shift
mkdir -p $out
KB=("$@")
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $out/$name -o $name -- \
      python tools/kbench.py --iters 2 "${KB[@]}" > $out/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY
run sq2 SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
run tcc TCC_HIT_sum TCC_MISS_sum
run fetch FETCH_SIZE
run write WRITE_SIZE
