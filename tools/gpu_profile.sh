#!/bin/bash
# rocprofv3 passes for the bench config (run on the GPU box from the repo root).
# Pass 1: kernel trace + stats.  Passes 2..: PMC counters, each its own run.
set -e
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
export GH_PROF_STEPS=${GH_PROF_STEPS:-100}  # the bench line's steps (and warm-up): kernel averages comparable
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 tools/profile_run.py > "$OUT/trace.log" 2>&1
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  GH_PROF_STEPS=10 timeout -k 10 240 rocprofv3 --pmc $ctrs -d "$OUT/pmc$i" -o run --output-format csv -- python3 tools/profile_run.py > "$OUT/pmc$i.log" 2>&1
done
