#!/bin/bash
# Repeat bench.py variants on one box (A/B without box-to-box noise):
#   tools/gpu_bench_rep.sh OUT REPS "args A" "args B" ...
# a variant "lib.so|args" runs bench.py with GEN_HIP_LIB=lib.so (another build);
# writes OUT/<i>_<rep>.json and a summary OUT/summary.txt (us per step).
set -e
OUT=$1; REPS=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in $(seq 1 "$REPS"); do
  i=0
  for args in "$@"; do
    i=$((i+1))
    lib=""
    if [[ "$args" == *"|"* ]]; then lib="${args%%|*}"; args="${args#*|}"; fi
    GEN_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline $args > "$OUT/${i}_${rep}.json" 2> "$OUT/${i}_${rep}.err"
  done
done
python - "$OUT" "$REPS" "$@" > "$OUT/summary.txt" <<'EOF'
import json, sys
out, reps, variants = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for i, v in enumerate(variants, 1):
    us = []
    for r in range(1, reps + 1):
        s = open(f"{out}/{i}_{r}.json").read()
        d = json.loads(s[s.index('{"metric"'):])  # (RCCL prints a banner first on the forced multi-rank path)
        us.append(d["ms_per_step"] * 1e3)
    print(f"{v!r:60s} us/step " + " ".join(f"{u:.2f}" for u in us) + f"  kernel_ms {d['roofline']['kernel_avg_ms']}")
EOF
cat "$OUT/summary.txt"
