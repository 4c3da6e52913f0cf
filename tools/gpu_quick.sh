#!/bin/bash
# Parity tests, the default bench line and a kernel-trace profile (no PMC).
set -e
mkdir -p gpurun_out/quick
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/quick/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/quick/bench.json 2> gpurun_out/quick/bench.err
GH_PROF_STEPS=20 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/quick/trace -o run --output-format csv -- python3 tools/profile_run.py > gpurun_out/quick/trace.log 2>&1
