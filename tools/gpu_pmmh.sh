#!/bin/bash
set -e
mkdir -p gpurun_out/pmmh
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pmmh/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/bench_pmmh.py > gpurun_out/pmmh/bench_pmmh.json 2> gpurun_out/pmmh/bench_pmmh.err
