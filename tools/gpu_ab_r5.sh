#!/bin/bash
# Round-5 A/B at the driver's bench configuration (--steps 20 --warmup 5), all
# variants interleaved on ONE box (the pool's box-to-box spread is larger than
# the effects):  HEAD (events on every step launch), HEAD --time-every 10,
# HEAD --no-kernel-timing, HEAD without the k_step block remap (variant
# build), and the round-3 tree (ab/r3, built from commit 615f75f).
#   tools/gpu_ab_r5.sh REPS [extra bench args]
set -e
REPS=${1:-4}; shift || true
EXTRA="$*"
OUT=$PWD/gpurun_out/ab_r5
mkdir -p $OUT
export TMPDIR=/tmp
B="--no-cpu-baseline --no-secondary --steps 20 --warmup 5 $EXTRA"
run() {  # name, then the command
  local name=$1; shift
  timeout -k 10 120 "$@" > $OUT/${name}_$rep.json 2> $OUT/${name}_$rep.err
}
for rep in $(seq 1 "$REPS"); do
  run head python bench.py $B
  run te10 python bench.py $B --time-every 10
  run notime python bench.py $B --no-kernel-timing
  GEN_HIP_LIB=$PWD/gen_amd/variants/noremap.so run noremap python bench.py $B
  (cd ab/r3 && run r3 python bench.py $B)
  echo "rep $rep done"
done
python - $OUT $REPS <<'EOF'
import json, sys, glob, statistics as st
out, reps = sys.argv[1], int(sys.argv[2])
for name in ["head", "te10", "notime", "noremap", "r3"]:
    us, ks = [], []
    for r in range(1, reps + 1):
        for path in (f"{out}/{name}_{r}.json",):
            try:
                s = open(path).read()
            except OSError:
                continue
            d = json.loads(s[s.index('{"metric"'):])
            us.append(d["ms_per_step"] * 1e3)
            ks.append(d["roofline"]["kernel_avg_ms"] * 1e3)
    if us:
        print(f"{name:8s} us/step " + " ".join(f"{u:.2f}" for u in us) + f"  median {st.median(us):.2f}"
              f"  k_step us " + " ".join(f"{k:.2f}" for k in ks))
EOF
