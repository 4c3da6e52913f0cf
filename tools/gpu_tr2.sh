#!/bin/bash
# The driver's multi-GPU launch rehearsed with 2 ranks on the one GPU of the
# box (peer transport with its probe, the default), then the same over RCCL
# is not possible (one device): the gloo-staged transport instead.
set -e
OUT=$PWD/gpurun_out/tr2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 2 --steps 20 --warmup 5 --particles 262144 > $OUT/tr2_peer.json 2> $OUT/tr2_peer.err
python -c "import json,sys; s=open('$OUT/tr2_peer.json').read(); j=json.loads(s[s.index('{\"metric\"'):]); print(j['value'], j['ms_per_step'], j['config']['transport'])"
grep -i "probe\|unavailable" $OUT/tr2_peer.err || true
