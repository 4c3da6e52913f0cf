#!/bin/bash
# One GPU session: parity tests, the default bench line, rocprofv3 passes.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
bash tools/gpu_profile.sh gpurun_out/prof
