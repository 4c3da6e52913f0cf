#!/bin/bash
# A/B: the current tree (variant base) against a library built from an
# earlier commit (variant prev), interleaved on one box, C2 and C4.
set -e
mkdir -p gpurun_out/abprev
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python tools/variants.py run base prev >> gpurun_out/abprev/c2.log 2>&1
  GH_VARIANT_ARGS="--steps 50 --model kitagawa --particles 2097152" timeout -k 10 300 python tools/variants.py run base prev >> gpurun_out/abprev/c4.log 2>&1
done
