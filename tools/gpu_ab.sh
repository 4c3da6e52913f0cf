#!/bin/bash
# A/B of the step kernels (pipelined default vs flat), after the GPU parity tests.
set -e
OUT=gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
for k in pipe flat pipe flat; do
  GH_STEP_KERNEL=$k timeout -k 10 300 python bench.py --no-cpu-baseline >> $OUT/c2_$k.jsonl 2>> $OUT/bench.err
  GH_STEP_KERNEL=$k timeout -k 10 300 python bench.py --no-cpu-baseline --model kitagawa --particles 2097152 >> $OUT/c4_$k.jsonl 2>> $OUT/bench.err
done
