#!/bin/bash
# flush A/B inside the 20-step bench: rounds of (default, exp libs...), flush_ms per run
# usage: tools/flush_ab.sh rounds name...
set -e
rounds=$1; shift
run() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-events none > gpurun_out/fab.log 2>&1
  echo "$label $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fab.log) $(grep -o '"flush_ms": [0-9.]*' gpurun_out/fab.log)"
}
for i in $(seq 1 "$rounds"); do
  run base X=0
  for v in "$@"; do run "$v" CTR_LIB_PATH=exp/lib_$v.so; done
done
