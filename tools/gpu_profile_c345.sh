#!/bin/bash
# rocprofv3 passes for the secondary configurations: C4 (Kitagawa PF, 2^21
# particles), C3 (coal RJMCMC) and C5 (PMMH): kernel trace + stats, then PMC
# groups (one per run): HBM bytes for the C4 step kernel, VALU/wave counters
# for all three.
set -e
OUT=${1:-gpurun_out/prof345}
mkdir -p "$OUT"
export TMPDIR=/tmp
C4="tools/profile_run.py --model kitagawa --particles 2097152"
C3="tools/bench_coal.py --cpu-chains 1"
C5="tools/bench_pmmh.py --cpu-chains 1 --iters 1"
i=0
for w in c4 c3 c5; do
  case $w in c4) cmd=$C4;; c3) cmd=$C3;; c5) cmd=$C5;; esac
  GH_PROF_STEPS=100 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/$w.trace" -o run --output-format csv -- python3 $cmd > "$OUT/$w.trace.log" 2>&1
  for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
              "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU" \
              "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    GH_PROF_STEPS=10 timeout -k 10 240 rocprofv3 --pmc $ctrs -d "$OUT/$w.pmc$i" -o run --output-format csv -- python3 $cmd > "$OUT/$w.pmc$i.log" 2>&1
  done
done
