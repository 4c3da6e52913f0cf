#!/bin/bash
# GPU tests of the tree, then an interleaved A/B of the tree's library against
# prev_lib.so (a library built from another commit, copied to the repo root).
set -e
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_gpu.log 2>&1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 > gpurun_out/ab/new_$i.json 2>/dev/null
  GEN_HIP_LIB=$PWD/prev_lib.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 > gpurun_out/ab/prev_$i.json 2>/dev/null
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 --model kitagawa --particles 2097152 > gpurun_out/ab/new_c4.json 2>/dev/null
GEN_HIP_LIB=$PWD/prev_lib.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 --model kitagawa --particles 2097152 > gpurun_out/ab/prev_c4.json 2>/dev/null
