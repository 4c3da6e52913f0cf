# bench.py's multi-rank branch as the driver launches it, 2 ranks on the one GPU (gloo transport: a plumbing rehearsal)
set -e
O=gpurun_out/tr2
mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --transport gloo --particles 262144 > $O/bench.json 2> $O/bench.err
