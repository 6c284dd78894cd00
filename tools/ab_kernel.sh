#!/bin/bash
# Isolated-kernel A/B on the GPU box: tools/kbench.py with the in-tree library and an experiment build
# (tools/build_exp.sh), alternated three times.  Usage: tools/ab_kernel.sh <exp lib name> <kbench args...>
name=$1; shift
for i in 1 2 3; do
  echo "== base $i"; timeout -k 10 120 python tools/kbench.py "$@" || exit 1
  echo "== $name $i"; CTR_LIB_PATH=exp/lib_$name.so timeout -k 10 120 python tools/kbench.py "$@" || exit 1
done
