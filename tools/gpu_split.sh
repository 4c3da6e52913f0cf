#!/bin/bash
# multi-rank GPU tests, the GPU suite, then base vs prev on C2 (four alternations) and C4
set -e
mkdir -p gpurun_out/split
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_multirank.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/split/pytest_multirank.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/split/pytest_gpu.log 2>&1
for i in 1 2 3 4; do
  timeout -k 10 300 python tools/variants.py run base prev >> gpurun_out/split/c2.log 2>&1
done
for i in 1 2; do
  GH_VARIANT_ARGS="--steps 50 --model kitagawa --particles 2097152" timeout -k 10 300 python tools/variants.py run base prev >> gpurun_out/split/c4.log 2>&1
done
