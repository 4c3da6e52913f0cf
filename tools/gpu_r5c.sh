#!/bin/bash
# Round-5 GPU pass C: GPU tests named in $1, then the resample's phase clocks
# at C4 with the pair kernel folding its maxima into the shards (variant).
set -e
OUT=$PWD/gpurun_out/r5c
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$1" ]; then
  timeout -k 10 1000 python -u -m pytest $1 -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  tail -3 $OUT/pytest.log
fi
GEN_HIP_LIB=$PWD/gen_amd/variants/rs_stamps.so timeout -k 10 120 python tools/rs_stamps.py lg10 20 > $OUT/rs_lg10.txt 2>&1
GEN_HIP_LIB=$PWD/gen_amd/variants/rs_stamps.so timeout -k 10 120 python tools/rs_stamps.py kit 21 > $OUT/rs_kit.txt 2>&1
cat $OUT/rs_lg10.txt $OUT/rs_kit.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
python - $OUT/bench.json <<'PY'
import json, sys
s = open(sys.argv[1]).read(); d = json.loads(s[s.index('{"metric"'):])
print("C2", d["ms_per_step"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"])
sec = d["secondary"]
print("C4", sec["C4"]["ms_per_step"], "cbc", json.dumps(sec["call_by_call"]))
print("mr", json.dumps(sec["multirank_path"]))
PY
