#!/bin/bash
# row-sharded tables under the reference's autograd loop (world 2 on one card over gloo)
set -e
mkdir -p gpurun_out/r05g
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05g/shard_autograd.log 2>&1 || { tail -n 60 gpurun_out/r05g/shard_autograd.log; exit 1; }
tail -n 3 gpurun_out/r05g/shard_autograd.log
