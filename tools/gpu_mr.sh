#!/bin/bash
set -e
mkdir -p gpurun_out/mr
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/mr/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/mr/bench.json 2> gpurun_out/mr/bench.err
