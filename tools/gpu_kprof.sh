#!/bin/bash
# Interleaved rocprofv3 kernel traces of library variants on one box (run on
# the GPU box from the repo root):
#   bash tools/gpu_kprof.sh OUTDIR REPS label=lib.so[@VAR=value] ...
# ("head" = the in-tree library).  C2 and C4 bench configs, GH_PROF_STEPS
# (default 30) steps each; prints per label the median over runs of each
# kernel's average duration and of the gaps between consecutive kernels.
set -e
OUT=$PWD/$1; REPS=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
export GH_PROF_STEPS=${GH_PROF_STEPS:-30}
for rep in $(seq 1 $REPS); do
  for m in "c2|" "c4|--model kitagawa --particles 2097152"; do
    name=${m%%|*}; args=${m#*|}
    for lv in "$@"; do
      label=${lv%%=*}; lib=${lv#*=}
      xenv=""; case "$lib" in *@*) xenv=${lib#*@}; lib=${lib%%@*};; esac
      (
        if [ "$lib" != "head" ]; then export GEN_HIP_LIB=$PWD/$lib; fi
        if [ -n "$xenv" ]; then export "$xenv"; fi
        timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/${name}_${label}_$rep -o run --output-format csv \
          -- python3 tools/profile_run.py $args > $OUT/${name}_${label}_$rep.log 2>&1
      )
    done
  done
done
python - $OUT $REPS "$@" <<'PY'
import csv, glob, sys, statistics as st
out, reps, labels = sys.argv[1], int(sys.argv[2]), [a.split("=")[0] for a in sys.argv[3:]]
def short(k):
    return k.split("(")[0].replace("void gh::", "").replace("gh::", "")
for name in ("c2", "c4"):
    for v in labels:
        per = {}
        gaps = {}
        for r in range(1, reps + 1):
            f = glob.glob(f"{out}/{name}_{v}_{r}/**/*kernel_trace.csv", recursive=True)
            rows = sorted(csv.DictReader(open(f[0])), key=lambda x: int(x["Start_Timestamp"]))
            rows = rows[len(rows) // 3:]  # (past the set-up and warm-up launches)
            d = {}
            g = {}
            for a, b in zip(rows, rows[1:]):
                g.setdefault(short(a["Kernel_Name"]) + "->" + short(b["Kernel_Name"]), []).append(
                    (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
            for x in rows:
                d.setdefault(short(x["Kernel_Name"]), []).append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
            for k, xs in d.items():
                per.setdefault(k, []).append(st.mean(xs))
            for k, xs in g.items():
                gaps.setdefault(k, []).append(st.mean(xs))
        print(name, v, "  ".join(f"{k} {st.median(xs):.2f}" for k, xs in sorted(per.items()) if len(xs) == reps),
              "| gaps", "  ".join(f"{k} {st.median(xs):.2f}" for k, xs in sorted(gaps.items()) if len(xs) == reps))
PY
