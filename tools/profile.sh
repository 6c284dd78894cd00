#!/bin/bash
# Profiling passes on the GPU box (run from the repo root through gpurun).  Every GPU step runs under its
# own time limit and the script stops at the first failure (set -e).  Outputs go to gpurun_out/<tag>/;
# copy the summaries that are judged into profiles/rNN/.
#
#   tools/profile.sh <tag> [steps...]
#     trace     rocprofv3 --kernel-trace --stats of a 20-step bench with step markers (tools/prof_summary.py
#               and tools/gap_summary.py summarise the timed steps)
#     pmc       one rocprofv3 --pmc pass per counter group (FETCH_SIZE / WRITE_SIZE separately, as
#               MI355X_MICROARCH.md prescribes), 3 timed steps with markers
#     pmc4      the same counter groups at --config cfg4
#     trace4    the kernel trace at --config cfg4 (6 timed steps)
#     bench     the default bench line (100 timed steps + CPU baseline) and the driver's 20 + 5
#     cfgs      cfg3 / cfg4 bench lines (parity configs, not the headline)
#   default: trace pmc bench
set -e
export TMPDIR=/tmp
tag=${1:?tag}
shift
steps=${*:-trace pmc bench}
out=gpurun_out/$tag
mkdir -p "$out"
pmc() {  # name config counters...
  local name=$1 cfg=$2
  shift 2
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$out/pmc_$name" -o "$name" -- \
      python bench.py --config "$cfg" --steps 3 --warmup 2 --no-cpu-baseline --no-fp32-secondary --markers > "$out/pmc_$name.log" 2>&1
}
pmc_groups() {  # suffix config
  pmc "fetch$1" "$2" FETCH_SIZE
  pmc "write$1" "$2" WRITE_SIZE
  pmc "valu$1" "$2" SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
  # f32 MFMA ops (the QNN Gram products, the fused layer forward's projections) in their own pass: the valu pass
  # holds 7 SQ counters already
  pmc "mops$1" "$2" SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE
  pmc "lds$1" "$2" SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU \
      SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY
}
for s in $steps; do
  case $s in
    trace)
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o trace -- \
          python bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-fp32-secondary --markers > "$out/trace.log" 2>&1 ;;
    pmc) pmc_groups "" cfg2 ;;
    pmc4) pmc_groups "_cfg4" cfg4 ;;
    trace4)
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace4" -o trace4 -- \
          python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline --no-fp32-secondary --markers > "$out/trace4.log" 2>&1 ;;
    bench)
      timeout -k 10 240 python bench.py > "$out/bench_n1.log" 2>&1
      timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$out/bench_n1_s20.log" 2>&1 ;;
    cfgs)
      timeout -k 10 200 python bench.py --config cfg3 --steps 10 --warmup 3 --no-cpu-baseline > "$out/bench_cfg3.log" 2>&1
      timeout -k 10 200 python bench.py --config cfg4 --steps 6 --warmup 3 --no-cpu-baseline > "$out/bench_cfg4.log" 2>&1 ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
