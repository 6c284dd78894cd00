#!/bin/bash
# flush A/B on the synthetic lazy state (tools/flushbench.py): default library vs exp/lib_<name>.so
# usage: tools/fb_ab.sh "<flushbench args>" name...
set -e
args=$1; shift
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L="exp/lib_$v.so"; fi
  echo "== $v ($args)"
  CTR_LIB_PATH=$L timeout -k 10 120 python tools/flushbench.py $args 2>&1 | grep -v amdgpu.ids
done
