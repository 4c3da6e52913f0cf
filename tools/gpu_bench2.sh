#!/bin/bash
# Rehearse the multi-rank bench flow on one GPU: 2 and 3 ranks over the gloo host transport.
set -e
mkdir -p gpurun_out/b2
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --transport gloo --particles 262144 --steps 10 --warmup 2 > gpurun_out/b2/bench2.json 2> gpurun_out/b2/bench2.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 3 --transport gloo --model kitagawa --particles 300000 --steps 10 --warmup 2 > gpurun_out/b2/bench3.json 2> gpurun_out/b2/bench3.err
