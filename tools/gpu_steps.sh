#!/bin/bash
# Run GPU steps in order on the gpurun box; each step has its own time limit.  A plain test failure
# (exit 1) lets later steps run; a crash / abort / timeout (any other non-zero code) stops the script.
# usage: tools/gpu_steps.sh "name:seconds:command" ...
set +e
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start )) s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping after [$name] (rc=$rc)"
    exit $rc
  fi
done
exit 0
