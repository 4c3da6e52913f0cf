# bench.py's multi-rank branch as the driver launches it, 2 ranks on the one GPU
# (a plumbing rehearsal: two processes share the device, so the step time says
# nothing about 2 GPUs).  TRANSPORT=peer|gloo|rccl (default peer).
set -e
O=${1:-gpurun_out/tr2}
T=${TRANSPORT:-peer}
mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --transport $T --particles 262144 > $O/bench_$T.json 2> $O/bench_$T.err
