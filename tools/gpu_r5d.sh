#!/bin/bash
# Round-5 GPU pass D: the driver's multi-GPU launch rehearsed with 2 ranks on
# the one GPU (peer transport, the new default), then an interleaved A/B of the
# block-wide carries (product vs GH_NO_HUGE_CARRIES) at C2 and C4, with the
# resample's phase clocks of both.
set -e
OUT=$PWD/gpurun_out/r5d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 2 --steps 20 --warmup 5 --particles 262144 > $OUT/tr2_peer.json 2> $OUT/tr2_peer.err
tail -c 400 $OUT/tr2_peer.json
for rep in 1 2 3 4; do
  for m in "c2|" "c4|--model kitagawa --particles 2097152"; do
    name=${m%%|*}; args=${m#*|}
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 5 $args > $OUT/${name}_head_$rep.json 2>/dev/null
    GEN_HIP_LIB=$PWD/gen_amd/variants/no_huge.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 5 $args > $OUT/${name}_nohuge_$rep.json 2>/dev/null
  done
done
for v in rs_stamps rs_stamps_nohuge; do
  GEN_HIP_LIB=$PWD/gen_amd/variants/$v.so timeout -k 10 120 python tools/rs_stamps.py lg10 20 > $OUT/${v}_lg10.txt 2>&1
  GEN_HIP_LIB=$PWD/gen_amd/variants/$v.so timeout -k 10 120 python tools/rs_stamps.py kit 21 > $OUT/${v}_kit.txt 2>&1
done
python - $OUT <<'PY'
import json, sys, statistics as st
out = sys.argv[1]
for name in ("c2", "c4"):
    for v in ("head", "nohuge"):
        us = []
        for r in range(1, 5):
            s = open(f"{out}/{name}_{v}_{r}.json").read()
            us.append(json.loads(s[s.index('{"metric"'):])["ms_per_step"] * 1e3)
        print(name, v, " ".join(f"{u:.2f}" for u in us), f"median {st.median(us):.2f}")
PY
tail -n 9 $OUT/rs_stamps_lg10.txt $OUT/rs_stamps_nohuge_lg10.txt $OUT/rs_stamps_kit.txt $OUT/rs_stamps_nohuge_kit.txt
