#!/bin/bash
# Functional rehearsal of the N=2 bench path on a one-card box: two ranks on one GPU over gloo (the
# collective sequence RCCL runs at N>1); timings from this are not performance numbers.
export CTR_DIST_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline
