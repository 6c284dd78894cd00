#!/bin/bash
# Kernel A/B experiments: builds exp/lib_<name>.so = libctrhip.so with one source recompiled under extra
# defines (e.g. tools/build_exp.sh ffn FFN_EXP=1 ffn.hip -DFFN_EXP=1).  Load one with CTR_LIB_PATH.
set -e
cd "$(dirname "$0")/../toss-next-ctr-prediction_amd"
name=$1; src=$2; shift 2
mkdir -p ../exp/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Wall -Wno-unused-function $([ "${EXP_REPLACES:-$src}" = attn_mf.hip ] && echo -mllvm -amdgpu-mfma-vgpr-form=1) "$@" \
    -c csrc/$src -o ../exp/obj/$name.o
objs=$(ls build/*.o | grep -v "build/${EXP_REPLACES:-$src}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../exp/lib_$name.so $objs ../exp/obj/$name.o
