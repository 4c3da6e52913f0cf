#!/bin/bash
# Round-5 GPU pass B: the peer-transport multi-process tests, the step
# kernel's block clocks, and an interleaved C4 A/B of variant libraries.
#   tools/gpu_r5b.sh "PYTEST ARGS" REPS VARIANT...
set -e
TESTS=$1; REPS=${2:-0}; shift 2 || true
OUT=$PWD/gpurun_out/r5b
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  tail -3 $OUT/pytest.log
fi
timeout -k 10 120 python tools/kstep_stamps.py 20 > $OUT/kstep_lg10.json 2> $OUT/kstep_lg10.err
cat $OUT/kstep_lg10.json
B="--no-cpu-baseline --no-secondary --steps 20 --warmup 5 --model kitagawa --particles 2097152"
for rep in $(seq 1 "$REPS"); do
  timeout -k 10 120 python bench.py $B > $OUT/ab_head_$rep.json 2> $OUT/ab_head_$rep.err
  for v in "$@"; do
    GEN_HIP_LIB=$PWD/gen_amd/variants/$v.so timeout -k 10 120 python bench.py $B > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err
  done
done
if [ "$REPS" -gt 0 ]; then
python - $OUT $REPS head "$@" <<'PY'
import json, sys, statistics as st
out, reps, names = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for name in names:
    us, ks = [], []
    for r in range(1, reps + 1):
        s = open(f"{out}/ab_{name}_{r}.json").read()
        d = json.loads(s[s.index('{"metric"'):])
        us.append(d["ms_per_step"] * 1e3)
        ks.append(d["roofline"]["kernel_avg_ms"] * 1e3)
    print(f"{name:12s} us/step " + " ".join(f"{u:.2f}" for u in us) + f"  median {st.median(us):.2f}"
          f"  k_step us " + " ".join(f"{k:.2f}" for k in ks), flush=True)
PY
fi
