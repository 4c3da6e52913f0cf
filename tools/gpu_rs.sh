#!/bin/bash
# resample phase clocks (GH_RS_STAMPS variant) for the C2 and C4 sizes
set -e
mkdir -p gpurun_out/rs
export TMPDIR=/tmp
timeout -k 10 120 python tools/rs_stamps.py lg10 20 > gpurun_out/rs/stamps_lg10.txt 2>&1
timeout -k 10 120 python tools/rs_stamps.py kit 21 > gpurun_out/rs/stamps_kit.txt 2>&1
if [ "$1" = "full" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rs/pytest_gpu.log 2>&1
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/rs/bench.json 2> gpurun_out/rs/bench.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --model kitagawa --particles 2097152 > gpurun_out/rs/bench_kit.json 2> gpurun_out/rs/bench_kit.err
fi
