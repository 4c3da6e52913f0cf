#!/bin/bash
# Interleaved A/B of bench.py step times on one box (run on the GPU box from
# the repo root):  bash tools/gpu_ab.sh OUTDIR REPS label=lib.so[@VAR=value] ...
# ("head" = the in-tree library; @VAR=value: an environment switch).  C2 and C4, the driver's --steps 20
# --warmup 5; prints per-label runs, median step time and step-kernel time.
# GH_AB_TESTS="pytest args" runs those GPU tests first; GH_AB_STAMPS=1 adds
# the resample phase clocks (gen_amd/variants/rs_stamps.so); GH_AB_ARGS adds
# bench arguments (e.g. --force-multirank); GH_AB_PMMH=1 times C5
# (tools/bench_pmmh.py) per label too; GH_AB_NO_PF=1 skips C2/C4.
set -e
OUT=$PWD/$1; REPS=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$GH_AB_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $GH_AB_TESTS -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
LABELS=""
CASES=("c2|" "c4|--model kitagawa --particles 2097152")
[ -n "$GH_AB_NO_PF" ] && CASES=()
for rep in $(seq 1 $REPS); do
  for m in "${CASES[@]}"; do
    name=${m%%|*}; args=${m#*|}
    for lv in "$@"; do
      label=${lv%%=*}; lib=${lv#*=}
      xenv=""; case "$lib" in *@*) xenv=${lib#*@}; lib=${lib%%@*};; esac  # label=lib@VAR=value
      if [ "$lib" = "head" ]; then env="$xenv"; else env="GEN_HIP_LIB=$PWD/$lib $xenv"; fi
      env $env timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 5 $GH_AB_ARGS $args > $OUT/${name}_${label}_$rep.json 2> $OUT/${name}_${label}_$rep.err
    done
  done
  if [ -n "$GH_AB_PMMH" ]; then
    for lv in "$@"; do
      label=${lv%%=*}; lib=${lv#*=}
      xenv=""; case "$lib" in *@*) xenv=${lib#*@}; lib=${lib%%@*};; esac
      if [ "$lib" = "head" ]; then env="$xenv"; else env="GEN_HIP_LIB=$PWD/$lib $xenv"; fi
      env $env timeout -k 10 120 python tools/bench_pmmh.py --cpu-chains 1 > $OUT/c5_${label}_$rep.json 2> $OUT/c5_${label}_$rep.err
    done
  fi
done
if [ -n "$GH_AB_STAMPS" ]; then
  GEN_HIP_LIB=$PWD/gen_amd/variants/rs_stamps.so timeout -k 10 120 python tools/rs_stamps.py lg10 20 > $OUT/rs_lg10.txt 2>&1
  GEN_HIP_LIB=$PWD/gen_amd/variants/rs_stamps.so timeout -k 10 120 python tools/rs_stamps.py kit 21 > $OUT/rs_kit.txt 2>&1
fi
python - $OUT $REPS "$@" <<'PY'
import json, sys, statistics as st
out, reps, labels = sys.argv[1], int(sys.argv[2]), [a.split("=")[0] for a in sys.argv[3:]]
import os
for name in ("c2", "c4"):
    if os.environ.get("GH_AB_NO_PF"):
        break
    for v in labels:
        us, ks = [], []
        for r in range(1, reps + 1):
            s = open(f"{out}/{name}_{v}_{r}.json").read()
            j = json.loads(s[s.index('{"metric"'):])
            us.append(j["ms_per_step"] * 1e3)
            ks.append(j["roofline"]["kernel_avg_ms"] * 1e3)
        print(name, v, " ".join(f"{u:.2f}" for u in us), f"median {st.median(us):.2f}", f"kernel {st.median(ks):.2f}")
if os.environ.get("GH_AB_PMMH"):
    for v in labels:
        ms = [json.loads(open(f"{out}/c5_{v}_{r}.json").read().strip().splitlines()[-1])["kernel_ms"] for r in range(1, reps + 1)]
        print("c5", v, " ".join(f"{m:.2f}" for m in ms), f"median kernel_ms {st.median(ms):.2f}")
PY
if [ -n "$GH_AB_STAMPS" ]; then grep -E "^(start|max|quantised|barrier|offsets|marks|end) " $OUT/rs_lg10.txt $OUT/rs_kit.txt; fi
