#!/bin/bash
set -e
mkdir -p gpurun_out/coal
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/coal/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/bench_coal.py > gpurun_out/coal/bench_coal.json 2> gpurun_out/coal/bench_coal.err
